#!/bin/bash
# Round-3 session g: the signature kernel without scratch (2 waves/SIMD, 248
# VGPRs; compile-time indices for the Q table) against the 3-wave build
# (lib_tx3: 452 B/lane of spills), with FETCH/WRITE_SIZE passes of both; then
# the whole GPU test suite on the product.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
TX3=$PWD/distributed-chess_amd/build/var/lib_tx3.so
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --only tx --no-cpu --tx-steps 3 > $O/bench_tx2w_$r.json 2>>$O/bench_tx.err || { tail $O/bench_tx.err; exit 1; }
  DCHESS_LIB=$TX3 timeout -k 10 200 python -u bench.py --only tx --no-cpu --tx-steps 3 > $O/bench_tx3w_$r.json 2>>$O/bench_tx.err || exit 2
done
for f in $O/bench_tx*w_?.json; do python -c "import json;d=json.load(open('$f'))['tx_signatures'];print('$f', {k: d[k] for k in d if k in ('value','kernel_ms','ms_per_step','kernel_avg_ms')})"; done
for v in 2w 3w; do
  L=""; [ $v = 3w ] && L=$TX3
  for c in FETCH_SIZE WRITE_SIZE; do
    DCHESS_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/txpmc_${v}_$c -o p -- python bench.py --only tx --no-cpu --tx-steps 1 --warmup 1 --steps 1 --profile-only > /dev/null 2>>$O/bench_tx.err || { tail $O/bench_tx.err; exit 3; }
  done
done
python - <<'PY'
import csv, glob
for v in ("2w", "3w"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = []
        for f in glob.glob(f"gpurun_out/txpmc_{v}_{c}/*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if "k_verify_tx" in r["Kernel_Name"]:
                    vals.append(float(r["Counter_Value"]))
        print(v, c, "per launch (KB):", [round(x) for x in vals])
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu_g.log 2>&1 || { tail -30 $O/pytest_gpu_g.log; exit 4; }
tail -3 $O/pytest_gpu_g.log
