#!/bin/bash
# Round-5 session L: the co-residency stress test, the live-validator tests
# (one resident wave per process, work stops it) and the replicas.
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stress.py tests/test_gpu_live.py tests/test_gpu_replicas.py > $O/pytest_l.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_l.log | tail -40
exit $rc
