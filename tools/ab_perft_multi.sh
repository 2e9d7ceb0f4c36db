#!/bin/bash
# Same-box A/B of several perft builds (VARS = names of distributed-chess_amd/build/var/lib_<name>.so;
# "prod" = the tree's libdchess.so), two alternating passes, bench.py --only perft (golden-checked).
VARS=${VARS:-"prod w3 s20 w5"}
for r in 1 2; do
  for v in $VARS; do
    L=$PWD/distributed-chess_amd/build/var/lib_$v.so; [ $v = prod ] && L=$PWD/distributed-chess_amd/libdchess.so
    DCHESS_LIB=$L timeout -k 10 120 python bench.py --only perft --no-cpu --steps 40 > gpurun_out/abm_$v$r.json 2> gpurun_out/abm_$v$r.err || { echo "run $v$r failed"; tail -3 gpurun_out/abm_$v$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abm_$v$r.json'));print('$v', round(d['ms_per_step']*1e3,1), round(d['kernels_ms_per_step']['count2']*1e3,1))"
  done
done
