#!/usr/bin/env python3
"""Two static checks of a kernel's private (scratch) memory use, on compiler
assembly (.s) or on the disassembly of a built library's code objects:

 (i)  bounds: every scratch_* access's highest byte (immediate offset + width,
      plus an SGPR base when the value of that SGPR can be traced to constants
      in the same block) must lie inside .private_segment_fixed_size; an
      access whose address is a VGPR or an untraceable SGPR is reported as
      unbounded, and so is a kernel with a dynamic stack;
 (ii) SGPR spills to VGPR lanes: a VGPR written by v_writelane_b32 holds
      spilled SGPRs in lanes that EXEC does not protect; any other write of
      that VGPR (a VALU result, a scratch reload) or a scratch store of it
      outside a whole-wave region (EXEC forced to -1) would lose or clobber
      inactive lanes -- reported per VGPR.

DESIGN.md section 3.6 records the outcome on the round-2 failing build
(k_count3c<1, 6144, 4> of commit 3d8df08 with -DDC_C2C_SOA=1) and on the
product; tests/test_spill_free.py runs it on the built library's kernels.

usage: scratch_bounds_check.py FILE.s|LIB.so [kernel-substring ...]
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
WIDTH = {"dword": 4, "dwordx2": 8, "dwordx3": 12, "dwordx4": 16, "short": 2, "byte": 1, "ushort": 2, "ubyte": 1,
         "sshort": 2, "sbyte": 1, "short_d16": 2, "short_d16_hi": 2, "byte_d16": 1, "byte_d16_hi": 1,
         "ubyte_d16": 1, "ubyte_d16_hi": 1, "sbyte_d16": 1, "sbyte_d16_hi": 1}
OFF = re.compile(r"offset:(-?\d+|0x[0-9a-fA-F]+)")
VREGS = re.compile(r"\bv\[?(\d+)(?::(\d+))?\]?")


def _int(x):
    return int(x, 16) if x.startswith("0x") else int(x)


def kernels_from_s(path):
    """{name: (lines, private_size, dynamic_stack)} from compiler assembly."""
    lines = open(path).read().split("\n")
    out, name, body = {}, None, []
    for ln in lines:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            name, body = m.group(1), []
            continue
        if name is None:
            continue
        if ln.startswith(".Lfunc_end"):
            priv = dyn = None
            for b in body:
                m = re.match(r"\s*\.amdhsa_private_segment_fixed_size\s+(\d+)", b)
                if m:
                    priv = int(m.group(1))
                m = re.match(r"\s*\.amdhsa_uses_dynamic_stack\s+(\d+)", b)
                if m:
                    dyn = int(m.group(1))
            out[name] = ([b.split(";")[0] for b in body], priv, bool(dyn))
            name = None
            continue
        body.append(ln)
    return out


def kernels_from_lib(path):
    """Same, from a shared library: code objects unbundled with llvm-objdump,
    metadata from the notes, instructions from the disassembly."""
    tmp = tempfile.mkdtemp()
    out = {}
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copy(path, lib)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", lib], cwd=tmp, check=True, capture_output=True)
        for f in sorted(os.listdir(tmp)):
            if not f.endswith("gfx950"):
                continue
            co = os.path.join(tmp, f)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            meta, name = {}, None
            for line in notes.splitlines():
                m = re.match(r"\s*\.name:\s+(\S+)", line)
                if m:
                    name = m.group(1)
                    meta[name] = [0, False]
                m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
                if m and name:
                    meta[name][0] = int(m.group(1))
                m = re.match(r"\s*\.uses_dynamic_stack:\s+(\S+)", line)
                if m and name:
                    meta[name][1] = m.group(1) == "true"
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout
            cur, body = None, []
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if m:
                    if cur in meta:
                        out[cur] = (body, meta[cur][0], meta[cur][1])
                    cur, body = m.group(1), []
                    continue
                body.append("\t" + line.split("//")[0].strip())
            if cur in meta:
                out[cur] = (body, meta[cur][0], meta[cur][1])
    finally:
        shutil.rmtree(tmp)
    return out


def split(ln):
    s = ln.strip()
    if not s or s.startswith(".") or s.endswith(":"):
        return None, []
    parts = s.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def check_kernel(lines, priv, dyn):
    """-> (bounds_findings, lane_spill_findings, n_scratch_ops, max_byte)"""
    bounds, lanes = [], []
    sval = {}  # SGPR -> constant within the current block
    n_ops, max_byte = 0, 0
    for ln in lines:
        if ln.strip().endswith(":"):
            sval.clear()
        mn, ops = split(ln)
        if mn is None:
            continue
        if mn in ("s_mov_b32", "s_movk_i32") and len(ops) == 2 and re.fullmatch(r"-?(\d+|0x[0-9a-fA-F]+)", ops[1]):
            sval[ops[0]] = _int(ops[1])
        elif mn in ("s_add_u32", "s_add_i32") and len(ops) == 3 and ops[1] in sval and re.fullmatch(
                r"-?(\d+|0x[0-9a-fA-F]+)", ops[2]):
            sval[ops[0]] = sval[ops[1]] + _int(ops[2])
        elif ops and ops[0] in sval and not mn.startswith(("s_cmp", "s_cbranch", "scratch_", "buffer_")):
            sval.pop(ops[0], None)
        if not mn.startswith("scratch_"):
            continue
        n_ops += 1
        w = WIDTH.get(mn.split("_", 2)[-1].replace("store_", "").replace("load_", ""))
        if w is None:
            w = WIDTH.get(mn.split("_")[-1], 4)
        m = OFF.search(ln)
        off = _int(m.group(1)) if m else 0
        store = "store" in mn
        vaddr = ops[0] if store else ops[1]
        saddr = ops[2] if len(ops) > 2 else "off"
        saddr = saddr.split()[0]
        base = 0
        if vaddr != "off":
            bounds.append(("unbounded (VGPR address)", ln.strip()))
            continue
        if saddr != "off":
            if saddr in sval:
                base = sval[saddr]
            else:
                bounds.append(("unbounded (SGPR base not traced)", ln.strip()))
                continue
        hi = base + off + w
        max_byte = max(max_byte, hi)
        if dyn:
            bounds.append(("dynamic stack", ln.strip()))
        elif priv is None or hi > priv or base + off < 0:
            bounds.append((f"bytes [{base + off}, {hi}) outside private_segment_fixed_size {priv}", ln.strip()))
    # (ii) SGPR-to-VGPR-lane spills
    # a VGPR holds SGPR spills when v_writelane writes it and nothing but
    # v_readlane reads it (a ballot word built with v_writelane and then
    # stored or combined is data, not a spill slot)
    spill_v = set()
    for ln in lines:
        mn, ops = split(ln)
        if mn == "v_writelane_b32" and ops:
            spill_v.add(ops[0])
    for ln in lines:
        mn, ops = split(ln)
        if mn is None or mn in ("v_writelane_b32", "v_readlane_b32") or not ops:
            continue
        srcs = ops[1:] if not mn.startswith(("scratch_store", "global_store", "buffer_store", "ds_write", "flat_store",
                                              "global_atomic", "ds_add", "ds_or")) else ops
        for o in srcs:
            for m in VREGS.finditer(o):
                a = int(m.group(1))
                b = int(m.group(2)) if m.group(2) else a
                for k in range(a, b + 1):
                    if f"v{k}" in spill_v and not mn.startswith("scratch_store"):
                        spill_v.discard(f"v{k}")
    if spill_v:
        wwm = False
        for ln in lines:
            mn, ops = split(ln)
            if mn is None:
                continue
            if mn in ("s_or_saveexec_b64", "s_mov_b64") and len(ops) == 2 and (
                    (mn == "s_or_saveexec_b64" and ops[1] == "-1") or (ops[0] == "exec" and ops[1] == "-1")):
                wwm = True
                continue
            if ops and ops[0] == "exec" and mn.startswith("s_"):
                wwm = False
            if mn in ("v_writelane_b32", "v_readlane_b32"):
                continue
            regs = set()
            if ops:
                for m in VREGS.finditer(ops[0] if not mn.startswith("scratch_store") else ops[1]):
                    a = int(m.group(1))
                    b = int(m.group(2)) if m.group(2) else a
                    regs |= {f"v{k}" for k in range(a, b + 1)}
            hit = regs & spill_v
            if hit and mn.startswith(("v_", "scratch_", "global_", "buffer_", "ds_", "flat_")) and not wwm:
                kind = "stored to scratch" if mn.startswith("scratch_store") else "written"
                lanes.append((f"SGPR-spill VGPR {sorted(hit)} {kind} under a possibly partial EXEC", ln.strip()))
    return bounds, lanes, n_ops, max_byte


def main():
    path = sys.argv[1]
    subs = sys.argv[2:]
    ks = kernels_from_lib(path) if path.endswith(".so") else kernels_from_s(path)
    bad = 0
    for name, (lines, priv, dyn) in sorted(ks.items()):
        if subs and not any(s in name for s in subs):
            continue
        b, l, n, mx = check_kernel(lines, priv, dyn)
        if n or l or b:
            print(f"{name[:90]}: private {priv} B, dynamic stack {dyn}, {n} scratch ops, highest byte {mx}, "
                  f"{len(b)} bounds finding(s), {len(l)} lane-spill finding(s)")
        for why, ln in (b + l)[:10]:
            print(f"    {why}: {ln}")
        bad += len(b) + len(l)
    print("findings", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
