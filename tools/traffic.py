#!/usr/bin/env python3
"""Per-launch DRAM traffic of the hot kernels from rocprofv3 PMC passes -> profiles/traffic.json.

usage: tools/traffic.py --tag r01 --fetch <FETCH_SIZE counter_collection.csv> --write <WRITE_SIZE csv>
                        [--stats <kernel_stats.csv>] [--out profiles/traffic.json]

FETCH_SIZE / WRITE_SIZE are derived counters in KiB per dispatch.  MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is
exact for 16 B/lane stores.  Both count L2 misses to the fabric (Infinity-Cache hits included), so they
are an upper bound on HBM bytes.  The ray/path streams of these kernels are 16 B/lane float4 loads and
stores (4 B/lane for slot/prim/dim, uncalibrated).
"""
import argparse
import collections
import csv
import json
from pathlib import Path

KERNELS = ("k_trace_closest", "k_path_shade", "k_generate", "k_path_film")


def kname(raw):
    base = raw.split("(")[0].replace("void ", "")
    base = base.split("<")[0]
    return base.split("::")[-1]


def per_dispatch(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        vals[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tag", required=True)
    p.add_argument("--fetch", required=True)
    p.add_argument("--write", required=True)
    p.add_argument("--stats")
    p.add_argument("--out", default="profiles/traffic.json")
    p.add_argument("--config", default="cornell", help="bench.py --config the PMC passes ran")
    a = p.parse_args()
    fetch = per_dispatch(a.fetch, "FETCH_SIZE")
    write = per_dispatch(a.write, "WRITE_SIZE")
    avg_ns = {}
    if a.stats:
        for r in csv.DictReader(open(a.stats)):
            avg_ns[kname(r["Name"])] = float(r["AverageNs"])
    out = {"tag": a.tag, "config": a.config, "units": "bytes per launch (mean over the run's dispatches)",
           "correction": "FETCH_SIZE x2 (gfx950 half-count of 16 B/lane reads), KiB -> bytes x1024",
           "kernels": {}}
    for k in KERNELS:
        if k not in fetch or k not in write:
            continue
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write[k]) / len(write[k])
        b = (2 * f + w) * 1024
        d = {"dispatches": len(fetch[k]), "fetch_kib_raw": round(f, 1), "write_kib": round(w, 1),
             "dram_bytes_per_launch": int(b)}
        if k in avg_ns:
            d["rocprof_avg_ns"] = round(avg_ns[k], 1)
            d["dram_gbs"] = round(b / avg_ns[k], 1)
        out["kernels"][k] = d
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
