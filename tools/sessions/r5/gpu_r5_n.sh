#!/bin/bash
# Round-5 session N: wave priority 3 in one window of the
# reproducer's instruction stream at a time, beside single-issue noise: the
# window whose priority removes the fault holds the vulnerable instructions.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
for v in t_prio_540_546 t_prio_546_552 t_prio_552_556 t_prio_555_559 t_prio_559_563 t_prio_563_567 t_prio_545_546 t_prio_555_558; do
  DC_DIAG_GRID=96 DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --ms 2500 --reps 2 --kinds=12 \
    >> $O/noise_n5.jsonl 2>> $O/noise_n5.err || exit 1
done
python -c "
import json
for l in open('$O/noise_n5.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-2], d['grid'], d['noise_kind'], d['diffs'])"
for v in t_prio_540_546 t_prio_546_552 t_prio_552_556 t_prio_555_559 t_prio_559_563 t_prio_563_567 t_prio_545_546 t_prio_555_558; do
done
python -c "
import json
    d=json.loads(l); print(d['lib'].split('/')[-2], d['grid'], d['noise_kind'], d['diffs'])"
