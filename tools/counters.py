#!/usr/bin/env python3
"""Per-launch PMC counters of the hot kernels -> profiles/counters_<config>.json (read by bench.py's roofline).

usage: tools/counters.py --config cfg3 --tag r02c --dir gpurun_out/cnt_cfg3_r02c [--out profiles/counters_cfg3.json]

The directory holds the single-lane (RTMI_LANES=1) rocprofv3 runs of `bench.py --config <config>` written by
scripts/gpu_counters.sh: kt/ (kernel trace stats), fetch/ (FETCH_SIZE), write/ (WRITE_SIZE), sq/ (SQ_INSTS_VALU and
the stall mix), each pass in a run of its own.  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the
bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores.  The guide
validates the doubling only for wide coalesced streaming reads, and these kernels also gather (sorted rays, slot
records, BVH lines), so every kernel also carries the undoubled figure (`dram_bytes_per_launch_raw`): the truth lies
between the two.  Both count
L2 misses to the fabric (Infinity-Cache hits included), so they bound HBM bytes from above.  SQ_INSTS_VALU counts
wave-level VALU instructions (one per wave64 instruction issued).
"""
import argparse
import collections
import csv
import glob
import json
from pathlib import Path

KERNELS = ("k_trace_closest", "k_trace_fallback", "k_path_shade", "k_path_shade_full", "k_path_shade_full_c1", "k_path_shade_full_c2",
           "k_bin_materials", "k_path_nee", "k_path_nee_fb", "k_path_shadow", "k_generate", "k_path_film",
           "k_ref_shade_film", "k_rs_hist", "k_rs_scatter", "k_rs_offsets", "k_rs_prep")
# the mixed-scene shade of one bounce with material bins: the binning pass and one kernel per material class, all
# inside the shade stage's HIP-event bracket (bench.py k_path_shade): summed per launch into "k_path_shade_full"
SHADE_BINNED = ("k_bin_materials", "k_path_shade_full_c1", "k_path_shade_full_c2")


def kname(raw):
    full = raw.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    base = full.split("<")[0].split("::")[-1]
    args = full.replace(" ", "").split("<")[1].rstrip(">").split(",") if "<" in full else []
    if base == "k_path_nee" and args[-1:] == ["true"]:
        return "k_path_nee_fb"  # the exact-traversal fallback instantiation (undecided vertices), not the NEE pass
    if base == "k_path_shade_full" and len(args) == 2 and args[1] in ("1", "2"):
        return base + "_c" + args[1]  # one material class's kernel (k_path_shade_full<Q, MC>)
    return base


def per_dispatch(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(str(Path(d) / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            vals[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", required=True)
    p.add_argument("--tag", required=True)
    p.add_argument("--dir", required=True)
    p.add_argument("--out")
    p.add_argument("--lib", default="computational_ray_tracer_amd/lib/librtmi355x.so",
                   help="the library build the runs used (its id is stamped into the output)")
    a = p.parse_args()
    d = Path(a.dir)
    fetch = per_dispatch(d / "fetch", "FETCH_SIZE")
    write = per_dispatch(d / "write", "WRITE_SIZE")
    sq = {c: per_dispatch(d / "sq", c) for c in ("SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES",
                                                  "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_WAVES")}
    tot_ns, calls = collections.Counter(), collections.Counter()  # instantiations of one name pooled
    for f in glob.glob(str(d / "kt" / "**" / "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            tot_ns[kname(r["Name"])] += float(r["TotalDurationNs"])
            calls[kname(r["Name"])] += int(r["Calls"])
    avg_ns = {k: tot_ns[k] / calls[k] for k in calls if calls[k]}
    import hashlib
    out = {"tag": a.tag, "config": a.config, "lanes": 1,
           "lib_sha16": hashlib.sha256(Path(a.lib).read_bytes()).hexdigest()[:16],
           "units": "per launch (mean over the run's dispatches); bytes; wave-level instructions",
           "correction": "dram_bytes_per_launch: FETCH_SIZE x2 (gfx950 half-count of 16 B/lane reads) + WRITE_SIZE; "
                         "dram_bytes_per_launch_raw: FETCH_SIZE x1 + WRITE_SIZE (the doubling is validated for wide "
                         "coalesced reads only); KiB -> bytes x1024",
           "kernels": {}}
    for k in KERNELS:
        e = {}
        if k in fetch and k in write:
            f = sum(fetch[k]) / len(fetch[k])
            w = sum(write[k]) / len(write[k])
            e.update(dispatches=len(fetch[k]), fetch_kib_raw=round(f, 1), write_kib=round(w, 1),
                     dram_bytes_per_launch=int((2 * f + w) * 1024), dram_bytes_per_launch_raw=int((f + w) * 1024))
        for c, v in sq.items():
            if k in v:
                e[c.lower() + "_per_launch"] = round(sum(v[k]) / len(v[k]), 1)
        if "sq_insts_valu_per_launch" in e:
            e["valu_insts_per_launch"] = e["sq_insts_valu_per_launch"]
        if k in avg_ns:
            e["rocprof_avg_ns"] = round(avg_ns[k], 1)
            if "dram_bytes_per_launch" in e:
                e["dram_gbs"] = round(e["dram_bytes_per_launch"] / avg_ns[k], 1)
        if e:
            out["kernels"][k] = e
    ks = out["kernels"]
    if all(k in ks for k in SHADE_BINNED) and "k_path_shade_full" not in ks:
        e = {"parts": list(SHADE_BINNED)}
        for f in ("dram_bytes_per_launch", "dram_bytes_per_launch_raw", "valu_insts_per_launch", "rocprof_avg_ns"):
            if all(f in ks[k] for k in SHADE_BINNED):
                e[f] = sum(ks[k][f] for k in SHADE_BINNED)
        if "dram_bytes_per_launch" in e and "rocprof_avg_ns" in e:
            e["dram_gbs"] = round(e["dram_bytes_per_launch"] / e["rocprof_avg_ns"], 1)
        ks["k_path_shade_full"] = e
    dst = Path(a.out or f"profiles/counters_{a.config}.json")
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
