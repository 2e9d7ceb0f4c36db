#!/bin/bash
# Full GPU parity suite on the product library, then the perft/replay bench legs
# with the fused final stage (default) and, in the A/B build, DC_FUSED3=0 (k_count2c).
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -u bench.py --no-cpu --only perft,perft6,perft8,replay > $O/bench_fused.json 2> $O/bench_fused.err || { tail $O/bench_fused.err; exit 2; }
DCHESS_LIB=$PWD/distributed-chess_amd/libdchess_ab.so DC_FUSED3=0 timeout -k 10 200 python -u bench.py --no-cpu --only perft,perft6 > $O/bench_c2c.json 2> $O/bench_c2c.err || { tail $O/bench_c2c.err; exit 3; }
python - <<'PY'
import json
for f in ("bench_fused", "bench_c2c"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    r = d.get("replay") or {}
    print(f, "perft7 %.4f ms %.3e" % (d["ms_per_step"], d["value"]), {k: round(v, 4) for k, v in d["kernels_ms_per_step"].items()},
          "perft6 %.4f" % d["perft6"]["ms_per_step"], "perft8 %s" % (d.get("perft8") or {}).get("ms_per_step"),
          "replay %s %s %s" % (r.get("ms_per_step"), r.get("kernel_avg_ms"), r.get("replay_parity")))
PY
