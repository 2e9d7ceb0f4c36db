#!/bin/bash
# Same-box A/B of the perft step between two builds of libdchess.so:
# A = $A (default: distributed-chess_amd/build/var/libprev.so), B = the tree's library.
# Alternates ABABAB (bench.py --only perft, 40 steps) and prints each step time;
# box-to-box variance (~1 %) is larger than the effects measured this way.
A=${A:-$PWD/distributed-chess_amd/build/var/libprev.so}
B=${B:-$PWD/distributed-chess_amd/libdchess.so}
for r in 1 2 3; do
  for v in A B; do
    L=$A; [ $v = B ] && L=$B
    DCHESS_LIB=$L timeout -k 10 120 python bench.py --only perft --no-cpu --steps 40 > gpurun_out/ab_$v$r.json 2>/dev/null || { echo "run $v$r failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));print('$v', round(d['ms_per_step']*1e3,1), {k: round(x*1e3,1) for k,x in d['kernels_ms_per_step'].items()})"
  done
done
