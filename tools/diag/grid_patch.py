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
# the REF final stage (k_count3c, dynamic groups: any grid is correct), if present
for stm in ("1", "0"):
    old = (f"    auto k = k_count3c<{stm}, kC3cCap, DC_C3C_MINW, W>;\n"
           f"    hipLaunchKernelGGL(k, dim3(resident_grid(k, 256, kMaxGrid)),")
    if old in s:
        s = s.replace(old, old.replace("resident_grid(k, 256, kMaxGrid)", "resident_grid(k, 256, diag_grid3())"))
if "diag_grid3()" in s:
    anchor = "template <class W>\nstatic hipError_t count3c_w("
    s = s.replace(anchor, "static u32 diag_grid3() {\n  const char* e = getenv(\"DC_DIAG_GRID3\");\n"
                          "  return e ? (u32)atoi(e) : kMaxGrid;\n}\n" + anchor, 1)
open(p, "w").write(s)
