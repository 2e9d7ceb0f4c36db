#!/bin/bash
# Round-5 session G: the reproducer's exact instruction
# stream with s_nop padding inserted at chosen places (tools/diag/asm_edit.py),
# run on 96 blocks beside single-issue noise (kind 12) and on the default grid.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
for v in t_asm_none t_asm_nopA1 t_asm_nopA4 t_asm_nopB4 t_asm_exec4 t_asm_vcmp4 t_asm_allv1 t_asm_gl4 t_asm_br4; do
  DC_DIAG_GRID=96 DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --ms 2500 --reps 2 --kinds=12 \
    >> $O/noise_g.jsonl 2>> $O/noise_g.err || exit 1
  DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --reps 2 --kinds=-1 \
    >> $O/noise_g.jsonl 2>> $O/noise_g.err || exit 1
done
python -c "
import json
for l in open('$O/noise_g.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-2], d['grid'], d['noise_kind'], d['diffs'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_live.py "tests/test_gpu_ref.py::test_perft6_ref_off_startpos_tree" > $O/pytest_g.log 2>&1 || { tail -30 $O/pytest_g.log; exit 1; }
tail -3 $O/pytest_g.log
