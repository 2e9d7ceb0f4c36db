#!/bin/bash
# Round-4 calibration session (run under gpurun from the repo root):
#   1. tools/ubench/dual_issue: SIMD cycles per wave64 instruction by class and
#      waves/SIMD (s_memtime), plain run and one PMC pass with the dual-issue
#      counter SQ_ACTIVE_INST_VALU2                      -> gpurun_out/r4/ubench_*
#   2. one PMC pass over the perft/replay/generator legs with the VALU issue
#      counters (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_VALU2,
#      wave/busy/wait cycles, GRBM_GUI_ACTIVE)          -> gpurun_out/r4/pmc_issue/
#   3. a default bench run (baseline of this round)    -> gpurun_out/r4/bench_base.json
# Every GPU step has its own limit; the first failure ends the script.
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
step() { echo "[$(date +%T)] $*" >> $O/steps.log; }
step ubench
timeout -k 10 120 ./tools/ubench/dual_issue > $O/ubench_dual_issue.txt 2>&1 || { tail $O/ubench_dual_issue.txt; exit 1; }
step ubench-pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/ubench_pmc -o p -- ./tools/ubench/dual_issue > /dev/null 2>> $O/pmc.err || { tail $O/pmc.err; exit 2; }
step pmc-issue
P="--steps 8 --warmup 1 --no-cpu --replay-steps 2 --only perft,replay"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_issue -o p -- python bench.py $P > /dev/null 2>> $O/pmc.err || { tail $O/pmc.err; exit 3; }
step live-tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_live.py tests/test_gpu_ref.py -x -v --timeout 120 --timeout-method thread > $O/pytest_live.log 2>&1 || { tail -30 $O/pytest_live.log; exit 6; }
tail -3 $O/pytest_live.log
step bench
timeout -k 10 400 python -u bench.py > $O/bench_base.json 2> $O/bench_base.err || { tail -20 $O/bench_base.err; exit 4; }
cat $O/bench_base.json
if [ -f distributed-chess_amd/build/bb/libdchess_bb.so ]; then
  step bbprof
  DCHESS_LIB=$PWD/distributed-chess_amd/build/bb/libdchess_bb.so timeout -k 10 120 python -u tools/bbprof_run.py perft7 $O/bbprof_count3c_d7.json 4 > $O/bbprof.log 2>&1 || { tail $O/bbprof.log; exit 5; }
  cat $O/bbprof.log
fi
step done
