#!/bin/bash
# Round 6, session 3: k_verify_tx with the owner comparison made before the
# message hash (strings read once): parity, FETCH/WRITE per launch, and the
# FETCH_SIZE calibration of the per-lane byte-load pattern (tools/ubench/fetch_calib.hip).
export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "txsig or tx_" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_tx_f -o p -- python bench.py --only tx --tx-steps 2 --no-cpu > /dev/null 2>> $O/pmc.err || { tail $O/pmc.err; exit 2; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_tx_w -o p -- python bench.py --only tx --tx-steps 2 --no-cpu > /dev/null 2>> $O/pmc.err || { tail $O/pmc.err; exit 3; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_calib -o p -- ./distributed-chess_amd/build/fetch_calib 262144 326 > $O/calib.json 2>> $O/pmc.err || { tail $O/pmc.err; exit 4; }
cat $O/calib.json
timeout -k 10 120 python -u bench.py --only tx --tx-steps 3 --no-cpu > $O/bench_tx.json 2> $O/bench.err || { tail $O/bench.err; exit 5; }
python - <<'PY'
import csv, collections
def agg(p, k):
    r = collections.defaultdict(list)
    for row in csv.DictReader(open(p)):
        if k in row["Kernel_Name"]:
            r[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {c: sum(v) / len(v) for c, v in r.items()}
O = "gpurun_out/r6d"
print("tx FETCH_SIZE KB", agg(O + "/pmc_tx_f/p_counter_collection.csv", "k_verify_tx"),
      "WRITE_SIZE KB", agg(O + "/pmc_tx_w/p_counter_collection.csv", "k_verify_tx"))
print("calib lane_bytes", agg(O + "/pmc_calib/p_counter_collection.csv", "k_lane_bytes"),
      "stream16", agg(O + "/pmc_calib/p_counter_collection.csv", "k_stream16"))
PY
echo done
