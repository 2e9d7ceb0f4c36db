#!/bin/bash
# Round-5 session M: the reproducer with its v_mov_b64 split
# into two v_mov_b32, and with padding before its global loads; the REF
# perft(6) off-startpos test.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
for v in t_asm_none t_asm_splitmov t_asm_bgl15; do
  DC_DIAG_GRID=96 DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --ms 2500 --reps 2 --kinds=12,1 \
    >> $O/noise_m.jsonl 2>> $O/noise_m.err || exit 1
  DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --reps 3 --kinds=-1 \
    >> $O/noise_m.jsonl 2>> $O/noise_m.err || exit 1
done
python -c "
import json
for l in open('$O/noise_m.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-2], d['grid'], d['noise_kind'], d['diffs'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_ref.py::test_perft6_ref_off_startpos_tree" > $O/pytest_m.log 2>&1; tail -3 $O/pytest_m.log
