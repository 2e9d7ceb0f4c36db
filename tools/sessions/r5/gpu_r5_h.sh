#!/bin/bash
# Round-5 session H: SGPR / EXEC padding variants of the
# reproducer beside single-issue noise; which call blocks behind a live wave.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
timeout -k 10 120 python -u tools/diag/live_block_probe.py >> $O/live_block_h.jsonl 2>&1 || exit 1
for v in t_asm_none t_asm_sdst15 t_asm_vcmp15 t_asm_exec15 t_asm_bexec15 t_asm_bsalu15 t_asm_exboth; do
  DC_DIAG_GRID=96 DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --ms 2500 --reps 2 --kinds=12 \
    >> $O/noise_h.jsonl 2>> $O/noise_h.err || exit 1
  DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --reps 2 --kinds=-1 \
    >> $O/noise_h.jsonl 2>> $O/noise_h.err || exit 1
done
cat $O/live_block_h.jsonl
python -c "
import json
for l in open('$O/noise_h.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-2], d['grid'], d['noise_kind'], d['diffs'])"
