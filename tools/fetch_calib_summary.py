#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE per access shape (scripts/gpu_calib.sh): counter bytes (KiB x 1024) over the bytes each
tools/fetch_calib.hip kernel moves, in launch order."""
import csv
import glob
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
shapes = [l.split() for l in open(str(d) + ".bytes.txt") if "_bytes" in l]
order = ["k_coalesced16", "k_gather", "k_gather", "k_gather", "k_store16", "k_scatter32"]


def per_launch(counter):
    rows = []
    for f in glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and r["Kernel_Name"].split("(")[0] in order:
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return [v for _, v in sorted(rows)]


fetch, write = per_launch("FETCH_SIZE"), per_launch("WRITE_SIZE")
rd32, rd = per_launch("TCC_EA0_RDREQ_32B_sum"), per_launch("TCC_EA0_RDREQ_sum")
out = {}
for i, s in enumerate(shapes):
    name, kv = s[0], dict(zip(s[1::2], (int(x) for x in s[2::2])))
    e = {"bytes": kv}
    if i < len(fetch):
        e["fetch_bytes"] = fetch[i] * 1024
        if "read_bytes" in kv:
            e["fetch_over_read"] = round(fetch[i] * 1024 / kv["read_bytes"], 3)
    if i < len(write):
        e["write_bytes"] = write[i] * 1024
        wb = kv.get("write_bytes", kv.get("sink_bytes", 0))
        if wb:
            e["write_over_bytes"] = round(write[i] * 1024 / wb, 3)
    if i < len(rd):
        e["rdreq"] = rd[i]
        e["rdreq_32b"] = rd32[i] if i < len(rd32) else None
    out[name] = e
print(json.dumps(out, indent=1))
