# One GPU round trip: parity tests, bench (no CPU legs), kernel-trace profile.
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --games 2000000 ${BENCH_ARGS} > /dev/null 2> gpurun_out/prof.err || exit 3
cat gpurun_out/bench.json
