"""Debug: dc_perft_repeat_device after torch CUDA init vs without (bench flow)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed-chess_amd"))
import dchess  # noqa: E402

mode = sys.argv[1]
depth = int(sys.argv[2])
steps = int(sys.argv[3])
if mode == "torch":
    import torch
    torch.cuda.synchronize()
eng = dchess.Engine(0)
s = dchess.startpos()
for _ in range(2):
    print("shard", eng.perft_shard(s, depth, 3, 0, 1)[0], flush=True)
if mode == "torch_late":
    import torch
    torch.cuda.synchronize()
buf = eng.alloc(steps * 258 * 8)
try:
    eng.perft_repeat_device(s, depth, 3, 0, 1, steps, buf)
    eng.synchronize()
    import numpy as np
    r = buf.download(np.uint64, steps * 258).reshape(steps, 258)
    print(mode, depth, steps, "ok", set(r[:, 257].tolist()), flush=True)
except Exception as e:
    print(mode, depth, steps, "FAIL", e, flush=True)
