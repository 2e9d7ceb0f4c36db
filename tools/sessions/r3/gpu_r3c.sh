#!/bin/bash
# Round-3 session c: final-stage child categories at perft(7) (A/B build,
# k_count2c PHASE 7: which of the opponent's slider groups a full-recount child
# changes), and the generator at 8 waves/SIMD (DC_GEN_MINW=8) against the
# product (7 waves).
set -o pipefail
O=gpurun_out
mkdir -p $O
AB=$PWD/distributed-chess_amd/libdchess_ab.so
DCHESS_LIB=$AB DC_FUSED3=0 DC_C2C_PHASE=7 DEPTH=7 timeout -k 10 120 python -u tools/c2c_stats.py > $O/c2c_stats_d7.txt 2>&1 || { cat $O/c2c_stats_d7.txt; exit 1; }
cat $O/c2c_stats_d7.txt
DCHESS_LIB=$AB DC_FUSED3=0 DC_C2C_PHASE=7 DEPTH=6 timeout -k 10 120 python -u tools/c2c_stats.py > $O/c2c_stats_d6.txt 2>&1 || exit 2
cat $O/c2c_stats_d6.txt
timeout -k 10 200 python -u bench.py --only replay --no-cpu --replay-steps 5 > $O/bench_gen_p.json 2>$O/bench_gen.err || { cat $O/bench_gen.err; exit 3; }
DCHESS_LIB=$PWD/distributed-chess_amd/build/var/lib_gen8.so timeout -k 10 200 python -u bench.py --only replay --no-cpu --replay-steps 5 > $O/bench_gen_8.json 2>>$O/bench_gen.err || exit 4
for v in p 8; do python -c "import json;d=json.load(open('$O/bench_gen_$v.json'))['replay'];print('$v', d['end_to_end']['ms_per_step'], d['end_to_end']['gen_kernel_avg_ms'], d['kernel_avg_ms'], d['replay_parity'])"; done
