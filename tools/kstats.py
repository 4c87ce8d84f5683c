#!/usr/bin/env python3
"""Per-kernel time table of a rocprofv3 --kernel-trace --stats run: python3 tools/kstats.py <kernel_stats.csv> [n]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms")
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", "")).replace("rtmi::", "")[-50:]
    print(f"{n:50s} {int(r['Calls']):5d} {float(r['TotalDurationNs']) / 1e6:8.2f} ms {float(r['AverageNs']) / 1e3:9.1f} us "
          f"{float(r['Percentage']):5.1f}%")
