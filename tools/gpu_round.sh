#!/bin/bash
# One full GPU round trip (run under gpurun from the repo root):
#   1. pytest -m gpu (parity)         -> gpurun_out/pytest_gpu.log
#   2. bench.py default (CPU legs on) -> gpurun_out/bench.json
#   3. rocprofv3 --kernel-trace --stats of the same bench (no CPU legs) -> gpurun_out/prof/
#   4. shard balance of perft(7)      -> gpurun_out/balance.jsonl
#   5. PMC passes (count2b + replay)  -> gpurun_out/pmc_*/ , gpurun_out/pmc_latest.json
# Every GPU step has its own time limit; the first failure ends the script.
export TMPDIR=/tmp
STAGES=${STAGES:-"test bench prof balance pmc"}
O=gpurun_out
has() { [[ " $STAGES " == *" $1 "* ]]; }
step() { echo "[$(date +%T)] $*" >> $O/steps.log; }
mkdir -p $O
if has test; then
  step pytest
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
if has bench; then
  step bench
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { cat $O/bench.err; exit 2; }
  cat $O/bench.json
fi
if has prof; then
  step prof
  rm -rf $O/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --no-cpu ${BENCH_ARGS} > $O/bench_prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 3; }
fi
if has balance; then
  step balance
  timeout -k 10 200 python -u tools/shard_balance.py 7 > $O/balance.jsonl 2>&1 || { cat $O/balance.jsonl; exit 4; }
fi
if has pmc; then
  # 4 counter passes over every leg's kernels (one bench process per pass),
  # then per-kernel records -> $O/pmc_latest.json (tools/pmc_summary.py)
  rm -rf $O/pmc_p*
  P="--steps 4 --warmup 1 --no-cpu --replay-steps 2 --hash-steps 1 --tx-steps 1 --only perft,perft8,perft9,replay,hash,tx"
  pass() {  # $1 counters, $2 tag
    step "pmc $2"
    timeout -s KILL 240 rocprofv3 --pmc $1 --output-format csv -d $O/pmc_$2 -o p -- python bench.py $P > /dev/null 2>> $O/pmc.err
  }
  pass "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" p1 && \
  pass "FETCH_SIZE" p2 && pass "WRITE_SIZE" p3 && \
  pass "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" p4 && \
  pass "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE" p5 || { tail $O/pmc.err; exit 5; }
  D8=$(python -c "import json;print(json.load(open('tests/golden/ref_deep.json'))['startpos_d8']['total'])")
  D9=$(python -c "import json;print(json.load(open('tests/golden/ref_deep.json'))['startpos_d9']['total'])")
  python tools/pmc_summary.py $O --json $O/pmc_latest.json --source "rocprofv3 --pmc (4 passes), bench.py $P" \
    --units "final_d7=k_count3c<0&unsigned int=3282734510" --units "final_d8=k_count3c<1&unsigned long=$D8" \
    --units "dfs_d9=k_perft_dfs<=$D9" \
    --units "replay=k_replay_ref4&true, false>=799999953" --units "gen_games=k_gen_games_ref=799999953" \
    --units "state_hash=k_state_hash_ref=1000000" --units "verify_tx=k_verify_tx=262144" > $O/pmc_summary.txt
fi
if has fidepmc; then
  # FIDE final stage (k_count2b<FideRules>): one bench process per leg so each
  # key's per-dispatch average comes from one workload; merged into pmc_latest.json
  rm -rf $O/pmc_f*
  for leg in fide7 fidesuite; do
    P="--steps 4 --warmup 1 --no-cpu --only $leg"
    [ $leg = fidesuite ] && P="$P --suite-batch-only"  # one kind of k_count2b dispatch: the six-position batch
    fpass() { local c=$1 t=$2; step "pmc $t"; timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$t -o p -- python bench.py $P > /dev/null 2>> $O/pmc.err; }
    fpass "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" f1$leg && \
    fpass "FETCH_SIZE" f2$leg && fpass "WRITE_SIZE" f3$leg && \
    fpass "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" f4$leg && \
    fpass "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE" f5$leg || { tail $O/pmc.err; exit 8; }
    mkdir -p $O/$leg && mv $O/pmc_f[1-5]$leg $O/$leg/
  done
  python tools/pmc_summary.py $O/fide7 --json $O/pmc_fide7.json --source "rocprofv3 --pmc (4 passes), bench.py --only fide7" \
    --units "fide_d7=k_count2b<dc::FideRules=3195901860" > $O/pmc_fide.txt
  python tools/pmc_summary.py $O/fidesuite --json $O/pmc_fidesuite.json --source "rocprofv3 --pmc (4 passes), bench.py --only fidesuite --suite-batch-only" \
    --units "fide_suite_d5=k_count2b<dc::FideRules=469080960" >> $O/pmc_fide.txt
  python - <<'PY'
import json, os
p = "gpurun_out/pmc_latest.json"
a = json.load(open(p)) if os.path.exists(p) else json.load(open("profiles/pmc_latest.json"))
for f in ("gpurun_out/pmc_fide7.json", "gpurun_out/pmc_fidesuite.json"):
    a.update(json.load(open(f)))
json.dump(a, open(p, "w"), indent=1)
PY
fi
if has txpmc; then
  rm -rf $O/pmc_t*
  P="--steps 1 --warmup 0 --no-cpu --profile-only --no-perft --no-replay --tx-steps 1"
  tpass() { local c=$1 t=$2; step "pmc $t"; timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$t -o p -- python bench.py $P > /dev/null 2>> $O/pmc.err; }
  tpass "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" t1 && \
  tpass "FETCH_SIZE" t2 && tpass "WRITE_SIZE" t3 && tpass "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" t4 && tpass "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE" t5 || { tail $O/pmc.err; exit 7; }
  mkdir -p $O/tx && mv $O/pmc_t[1-5] $O/tx/
  python tools/pmc_summary.py $O/tx --json $O/pmc_tx.json --units "verify_tx=k_verify_tx=262144" --source "rocprofv3 --pmc, bench.py $P" > $O/pmc_tx.txt
  python - <<'PY'
import json, os
p = "gpurun_out/pmc_latest.json"
a = json.load(open(p)) if os.path.exists(p) else json.load(open("profiles/pmc_latest.json"))
a.update(json.load(open("gpurun_out/pmc_tx.json")))
json.dump(a, open(p, "w"), indent=1)
PY
fi
step done
