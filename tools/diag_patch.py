"""Insert the DC_DIAG_CHILD per-child records (see dc_perft.hip, k_count2b) into
an older revision's dc_perft.hip (diagnostics for DESIGN.md §3.6; used as
PATCH="python tools/diag_patch.py distributed-chess_amd/csrc/dc_perft.hip"
with tools/ab_build_rev.sh).  The record code is copied from the working
tree, so both builds write the same records."""
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
wt = open(os.path.join(REPO, "distributed-chess_amd", "csrc", "dc_perft.hip")).read()
path = sys.argv[1]
src = open(path).read()
if "DC_DIAG_CHILD" in src:
    sys.exit(0)
decl = wt[wt.index("// DC_DIAG_CHILD (diagnostic builds only"):wt.index("template <class R, int STM>\n__global__ __launch_bounds__(256, R::kFinalMinBlocks) void k_count2b")]
rec = wt[wt.index("#ifdef DC_DIAG_CHILD\n          {"):]
rec = rec[:rec.index("#endif\n        }\n      }\n    }") + len("#endif\n")]
m = re.search(r"template <class R, int STM>\n__global__ __launch_bounds__\(256[^\n]*k_count2b", src)
src = src[:m.start()] + decl + src[m.start():]
body = src[m.start() + len(decl):]
i = body.index("  for (u64 s = blo; s < bhi; s += kChunk) {")
body = body[:i] + "#ifdef DC_DIAG_CHILD\n  u64 diag_off = (u64)blockIdx.x * per * 218;\n#endif\n" + body[i:]
anchor = "          else if (k) atomicAdd((unsigned long long*)&sh.hist[ptag], (unsigned long long)k);\n"
i = body.index(anchor) + len(anchor)
body = body[:i] + rec + body[i:]
anchor = "    tag_hist_add(sh.hist, tag0, acc, true);"
i = body.index(anchor)
body = body[:i] + "#ifdef DC_DIAG_CHILD\n    diag_off += total;\n#endif\n" + body[i:]
src = src[:m.start() + len(decl)] + body
open(path, "w").write(src)
