"""Per-kernel VGPRs / scratch / occupancy from hipcc's kernel-resource-usage
remarks (stdin), one line per kernel: python tools/res_report.py [filter] < remarks"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('vgpr', '?'):>4} vgpr {r.get('scratch', '?'):>4} B scratch {r.get('occ', '?')} w/SIMD "
              f"{r.get('lds', '?'):>6} B LDS  {r['name'].split('(')[0][:90]}")
