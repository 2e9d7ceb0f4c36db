#!/bin/bash
# Round-5 session O: at the fault site (v_cmp_ne_u64_e32 vcc,
# 0, v[102:103]; v_lshlrev_b64 v[106:107]; v_lshlrev_b64 v[102:103]) a VALU
# reader of VCC inserted after the compare, or s_nop 7 after it.
O=gpurun_out/r5
V=$PWD/distributed-chess_amd/build/var
mkdir -p $O
for v in t_prio_555_556 t_prio_556_557 t_prio_557_558 t_prio_556_558; do
  DC_DIAG_GRID=96 DCHESS_LIB=$V/$v/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --ms 2500 --reps 2 --kinds=12 >> $O/noise_o2.jsonl 2>> $O/noise_o2.err || exit 1
done
python -c "
import json
for l in open('$O/noise_o2.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-2], d['grid'], d['noise_kind'], d['diffs'])"
# the product's final stages on one block per CU (96 blocks) beside the noise
DC_DIAG_GRID=96 DCHESS_LIB=$V/prod_grid/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --ms 2500 --reps 2 --kinds=12,1,6 >> $O/noise_o3.jsonl 2>> $O/noise_o2.err || exit 1
DC_DIAG_GRID3=96 DCHESS_LIB=$V/prod_grid/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --rules ref --depth 7 --reps 6 --ms 4000 --kinds=12,1,6 >> $O/noise_o3.jsonl 2>> $O/noise_o2.err || exit 1
DC_DIAG_GRID3=96 DCHESS_LIB=$V/prod_grid/libdchess.so timeout -k 10 200 python -u tools/diag/noise_check.py --rules ref --depth 6 --reps 10 --ms 3000 --kinds=12,1 >> $O/noise_o3.jsonl 2>> $O/noise_o2.err || exit 1
python -c "
import json
for l in open('$O/noise_o3.jsonl'):
    d=json.loads(l); print(d['lib'].split('/')[-2], d['rules'], d['depth'], d['noise_kind'], d['victim_s'], d['diffs'])"
timeout -k 10 200 python -u tools/suite_time.py >> $O/suite_o.jsonl 2>> $O/suite_o.err || exit 1
for g in 768 384 256 1536; do
  DC_DIAG_GRID=$g DCHESS_LIB=$V/prod_grid/libdchess.so timeout -k 10 200 python -u tools/suite_time.py >> $O/suite_o.jsonl 2>> $O/suite_o.err || exit 1
done
cat $O/suite_o.jsonl
