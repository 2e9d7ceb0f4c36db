#!/bin/bash
# Round 6, session 3, final tree: smoke, then tools/gpu_round.sh's stages
# (the whole GPU suite, the default bench, its kernel trace, the PMC passes).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 12; }
tail -1 gpurun_out/smoke.log
STAGES="test bench prof pmc" bash tools/gpu_round.sh
