#!/usr/bin/env python3
"""Per-kernel resource table (VGPRs, spill bytes, occupancy, LDS) from hipcc -Rpass-analysis=kernel-resource-usage
remarks on stdin: `make -s resources | python3 tools/kres.py [filter]`."""
import re
import subprocess
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        name = re.sub(r"\(.*", "", name).replace("rtmi::", "")
        cur = {"name": name}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("spill", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r['name']:<48} vgpr {r.get('vgpr', '?'):>4} spill {r.get('spill', '?'):>4} occ {r.get('occ', '?'):>2} "
              f"lds {r.get('lds', '?'):>6}")
