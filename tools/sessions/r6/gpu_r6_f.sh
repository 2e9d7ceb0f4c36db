#!/bin/bash
# Round 6, session 3: the generator A/B (gpu_r6_e.sh), then the whole GPU
# suite and smoke on the product build.
export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
bash tools/sessions/r6/gpu_r6_e.sh || exit $?
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_full.log 2>&1 || { tail -30 $O/pytest_gpu_full.log; exit 11; }
tail -2 $O/pytest_gpu_full.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 12; }
tail -3 $O/smoke.log
echo done
