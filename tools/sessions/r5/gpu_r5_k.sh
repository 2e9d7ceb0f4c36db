#!/bin/bash
# Round-5 session K: which HIP call blocks behind the resident live waves
# (tests/test_gpu_live.py::test_live_waves_do_not_block_buffer_growth).
O=gpurun_out/r5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
true
timeout -k 10 400 rocprofv3 --hip-trace --output-format csv -d $O/livetrace -o live -- python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_live.py > $O/pytest_k_trace.log 2>&1
tail -3 $O/pytest_k_trace.log
F=$(find $O/livetrace -name "*hip_api_trace.csv" | head -1)
python - "$F" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), reverse=True)
for r in rows[:16]:
    print(r["Function"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9, r.get("Thread_Id"))
PY
rm -rf $O/livetrace
