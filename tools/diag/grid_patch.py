"""Host-only patch for an older revision's dc_perft.hip (diagnostics, DESIGN.md
§3.6): the FIDE final stage's grid from DC_DIAG_GRID (blocks), so a failing
kernel can run on a chosen number of blocks without a CU mask.  The kernels'
code is unchanged (tools/isa_norm_diff.py checks it)."""
import sys

p = sys.argv[1]
s = open(p).read()
old = "  else DC_LAUNCH_STM(k_count2b, FideRules, kMaxGrid, 256, st, nodes, meta, tags, rng, divide);"
assert old in s
s = s.replace(old, "  else DC_LAUNCH_STM(k_count2b, FideRules, diag_grid(), 256, st, nodes, meta, tags, rng, divide);")
anchor = "hipError_t launch_final("
s = s.replace(anchor, "static u32 diag_grid() {\n  const char* e = getenv(\"DC_DIAG_GRID\");\n"
                      "  return e ? (u32)atoi(e) : kMaxGrid;\n}\n" + anchor, 1)
open(p, "w").write(s)
