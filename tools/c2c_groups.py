"""Per-group leaf counts of k_count3c (builds with -DDC_C3C_LOG=1, see
tools/c2c_variants.sh): perft(startpos, d) through DCHESS_LIB, then the
per-group histogram log, differenced per block, saved as one row per group
(group, block, clock, leaves per root tag) to gpurun_out/groups_<TAG>_d<d>_r<run>.npy.
GPU tool: TAG=soa_log DCHESS_LIB=... python tools/c2c_groups.py 6 3"""
import ctypes, os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.getcwd(), "distributed-chess_amd"))
import dchess
d = int(sys.argv[1]); runs = int(sys.argv[2])
tag = os.environ.get("TAG", "x")
e = dchess.Engine(0)
lib = dchess.lib()
lib.dc_ab_c3c_log.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
G, W = 20480, 258
for r in range(runs):
    buf = np.zeros(G * W, np.uint64)
    lib.dc_ab_c3c_log(buf.ctypes.data, buf.size)   # clear? no: read stale, then overwrite below
    tot = e.perft(dchess.startpos(), d)[0]
    assert lib.dc_ab_c3c_log(buf.ctypes.data, buf.size) == 0
    rec = buf.reshape(G, W)
    # groups of this run: rows whose clock is newer than the run start
    n_groups = 1024 if d <= 6 else G  # perft(6): 771 groups
    np.save(f"gpurun_out/groups_{tag}_d{d}_r{r}.npy", rec[:n_groups])
    print(json.dumps({"tag": tag, "depth": d, "run": r, "total": int(tot)}), flush=True)
