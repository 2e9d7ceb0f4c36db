#!/bin/bash
# Round-5 session J: wave priority and region-restricted
# padding on the reproducer beside noise; the live-validator growth test.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
for v in t_asm_none t_asm_prio3 t_asm_cnt_v1 t_asm_out_v1; do
  DC_DIAG_GRID=96 DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --ms 2500 --reps 2 --kinds=12 \
    >> $O/noise_j.jsonl 2>> $O/noise_j.err || exit 1
  DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --reps 2 --kinds=-1 \
    >> $O/noise_j.jsonl 2>> $O/noise_j.err || exit 1
done
python -c "
import json
for l in open('$O/noise_j.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-2], d['grid'], d['noise_kind'], d['diffs'])"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_live.py > $O/pytest_j.log 2>&1; tail -15 $O/pytest_j.log
