#!/usr/bin/env python3
"""Per-bounce breakdown of a single-lane (RTMI_LANES=1) bench run: kernel time per depth from a rocprofv3 kernel
trace, and (optionally) per-dispatch PMC counters of the same depth from a counter-collection CSV of another run of
the same command (dispatch order is deterministic, so the n-th dispatch of a kernel is the same launch).

usage: tools/kdepth.py <kt_kernel_trace.csv> [pmc_counter_collection.csv ...]

A batch is k_generate, then per depth [sort kernels] k_trace_closest, the shade kernel(s) [sort, k_path_nee ...], and
k_path_film; the depth of a dispatch is the number of k_trace_closest dispatches since the last k_generate, minus 1.
"""
import collections
import csv
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    base = n.split("<")[0].split("::")[-1]
    args = n.split("<", 1)[1].rstrip(">").replace(" ", "") if "<" in n else ""
    if base == "k_path_nee" and args.endswith("true"):
        return "k_path_nee_fb"
    if base == "k_path_shade_full" and args[-2:] in (",1", ",2"):
        return base + "_c" + args[-1]
    return base


def walk(rows):
    """(kernel, depth) per dispatch, in dispatch order"""
    depth, out = -1, []
    for r in rows:
        k = short(r["Kernel_Name"])
        if k.startswith("__amd") or k.startswith("k_oct"):
            out.append((k, None))
            continue
        if k == "k_generate":
            depth = -1
        elif k == "k_trace_closest":
            depth += 1
        out.append((k, "film" if k == "k_path_film" else ("gen" if k == "k_generate" else depth)))
    return out


def main():
    kt = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Dispatch_Id"]))
    tags = walk(kt)
    dur = collections.defaultdict(list)
    for r, (k, d) in zip(kt, tags):
        if d is not None:
            dur[(k, d)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sys.argv[2:]:
        per = collections.defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(f)):
            i = int(r["Dispatch_Id"])
            per[i][r["Counter_Name"]] = float(r["Counter_Value"])
            names[i] = r
        rows = [names[i] for i in sorted(names)]
        for r, (k, d) in zip(rows, walk(rows)):
            if d is not None:
                for c, v in per[int(r["Dispatch_Id"])].items():
                    pmc[(k, d)][c].append(v)
    tot = sum(sum(v) for v in dur.values())
    print(f"{'kernel':<22} {'depth':>5} {'calls':>5} {'avg us':>9} {'share':>6}  counters (mean per dispatch)")
    order = {"gen": -2, "film": 99}
    for (k, d) in sorted(dur, key=lambda x: (order.get(x[1], x[1]), x[0])):
        v = dur[(k, d)]
        cs = {c: round(sum(x) / len(x) / 1e6, 1) for c, x in sorted(pmc[(k, d)].items())}
        print(f"{k:<22} {str(d):>5} {len(v):>5} {sum(v) / len(v):>9.1f} {100 * sum(v) / tot:>5.1f}%  "
              + (" ".join(f"{c}={x}M" for c, x in cs.items()) if cs else ""))


if __name__ == "__main__":
    main()
