#!/usr/bin/env python3
"""Benchmark: Msamples/s (whole node) of the MI355X path tracer on BASELINE.json configs[1] —
Cornell box, 1920x1080, 256 spp (16x16 stratified, jittered), diffuse + NEE, max depth 5.

One *step* = every GPU renders its pixel tiles (32x32 tiles, tile t -> rank t % N) for `spp_per_step * N`
sample indices, accumulating into its device-resident film; when a step completes the frame (256 indices) the
N films are reduced to rank 0 with one RCCL reduce over xGMI and the accumulation restarts.  Per-GPU work per step is fixed (weak scaling): W*H*spp_per_step samples.

Prints ONE JSON line on rank 0 (contract in the task statement): metric/value/unit, roofline of the dominant
kernel (by HIP-event time; algorithmic bytes per SURVEY.md §8(d) / its average launch time),
and the CPU baseline (the oracle's C++ restatement on host cores, bounded sample, N=1 rank 0 only).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from computational_ray_tracer_amd import capi, scene  # noqa: E402
from computational_ray_tracer_amd.distributed import FrameLoop, init_distributed, timed_steps  # noqa: E402
from computational_ray_tracer_amd.renderer import Renderer  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every 2 cycles at 2.4 GHz
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles (32 lanes/cycle x 2)")
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2
COUNTERS_DIR = ROOT / "profiles"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--warmup", type=int, default=1)
    # default: two lanes x one batch each at 1080p — 16 indices (16 Mi-sample batches) on the single-leaf Cornell box,
    # 32 (32 Mi) on the multi-level scenes (rt_host.cpp batch size)
    p.add_argument("--spp-per-step", type=int, default=None)
    p.add_argument("--res", type=str, default="1920x1080")
    p.add_argument("--config", choices=["cornell", "cfg3", "cfg4", "cfg5"], default="cornell",
                   help="cornell = BASELINE configs[1] (the metric's workload); cfg3..cfg5 = configs[2..4]")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-single-lane", action="store_true",
                   help="profiling runs only: skip the single-lane pass (no per-kernel roofline in the line)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    p.add_argument("--project-shards", type=int, default=8,
                   help="N=1 only: render each of the N pixel-tile shards of an N-GPU run on this GPU alone and project "
                        "the tile-parallel efficiency at N GPUs (0: off)")
    a = p.parse_args()
    if a.spp_per_step is None:
        a.spp_per_step = 16 if a.config == "cornell" else 32
    return a


def kernel_rooflines(st, counters, shadow_kernel="k_path_nee", sorted_bounces=False, n_lights=1):
    """Per-kernel HBM and VALU rooflines from HIP-event launch times (the single-lane pass: one launch at a time).

    Algorithmic bytes follow SURVEY.md §8(d): the per-ray HBM streams are `achieved` (k_trace_closest: 40 B per
    ray cast; k_path_shade: 312 B per shaded bounce + 32 B per shadow ray); the §8(d) scene terms (32 B per box
    test + 40 B per triangle test actually executed) are reported beside them as bytes only — they are cache hits
    (the Cornell scene is 1.8 KB, the CFG3 BVH 1 MB + 4.7 MB of triangles), never an HBM rate.  `traffic` is the
    PMC-measured DRAM bytes per launch and `valu` the SQ_INSTS_VALU per launch over the same single-lane launch time,
    both from profiles/counters_<config>.json when it was measured on the loaded library build."""
    # Multi-level scenes sort their bounce rays: the trace kernel reads each bounce ray through the
    # sort's permutation (4 B index) and writes it to the sorted side queue (32 B) on its way to the traversal —
    # the sort's data movement, fused into the trace: 36 B per bounce ray on top of the §8(d) 40 B.  (Gathering the
    # rays in the sort's last pass instead measured CFG3 -7 %, r04: the random reads are exposed there.)
    gather = 36 * max(0, st["rays"] - st["samples"]) if sorted_bounces else 0
    ks = {
        "k_trace_closest": (st["ms_trace"], st["launches_trace"], 40 * st["rays"] + gather,
                            32 * st["nodes_tested"] + 40 * st["tris_tested"]),
        "k_path_shade": (st["ms_shade"], st["launches_shade"], 312 * st["rays"] + 32 * st["shadow_rays"],
                         32 * st["shadow_nodes_tested"] + 40 * st["shadow_tris_tested"]),
    }
    # Multi-level simple path without the shadow queue: k_path_shade traces its shadow rays inline and k_path_shadow
    # only gets the few the BVH alone cannot decide (rt_kernels.hip k_path_shade), so the shadow bytes stay with the
    # shade kernel and the fallback kernel is reported by time only (its ray count is not counted on its own).
    fallback_only = shadow_kernel == "k_path_shadow" and os.environ.get("RTMI_SHADOW_QUEUE", "0") in ("", "0")
    fallback = None
    if st["ms_shadow"] > 0 and fallback_only:
        fallback = {"kernel": shadow_kernel, "role": "exact traversal of the undecided shadow rays only",
                    "launches": max(1, st["launches_shade"]),
                    "avg_launch_ms": round(st["ms_shadow"] / max(1, st["launches_shade"]), 4),
                    "total_ms": round(st["ms_shadow"], 3)}
    elif st["ms_shadow"] > 0:  # shadow rays in a kernel of their own, one launch per shade launch: the §8(d) 32 B
        # per shadow ray and the shadow scene terms move to it (k_path_nee: mixed scenes; k_path_shadow: shadow queue)
        # k_path_nee also reads each vertex's NEE record once (rt_internal.h NeeIO: po + material 16 B, the light
        # samples 8 B and weights 4 B per light: 64 B with 4 lights) and the slot's λ, β, L (96 B), and writes L and
        # β (64 B); vertices counted on the device (rt_stats nee_vertices)
        rec = 16 * (1 + (n_lights + 1) // 2 + (n_lights + 3) // 4) + 96 + 64
        ks[shadow_kernel] = (st["ms_shadow"], st["launches_shade"],
                             32 * st["shadow_rays"] + (rec * st.get("nee_vertices", 0)
                                                       if shadow_kernel == "k_path_nee" else 0),
                             32 * st["shadow_nodes_tested"] + 40 * st["shadow_tris_tested"])
        ks["k_path_shade"] = (st["ms_shade"], st["launches_shade"], 312 * st["rays"], 0)
    res = {}
    for name, (ms, launches, stream_b, scene_b) in ks.items():
        if ms <= 0:  # (a stage that did not run)
            continue
        launches = max(1, launches)
        avg_s = ms / launches * 1e-3
        a = stream_b / launches / avg_s / 1e9
        kc = (counters or {}).get(name) or (counters or {}).get(name + "_full", {})  # mixed scenes: k_path_shade_full
        res[name] = {"bound": "hbm", "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(a / HBM_PEAK_GBS, 4),
                     "traffic": kc.get("dram_bytes_per_launch"),
                     # FETCH_SIZE not doubled (the guide validates the x2 only for wide coalesced reads)
                     "traffic_raw": kc.get("dram_bytes_per_launch_raw"),
                     "kernel": name, "launches": launches, "avg_launch_ms": round(avg_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": int(stream_b / launches),
                     # §8(d) scene terms over the EXECUTED box / triangle tests: served by LDS / L1 / L2 (the
                     # scenes are <= 6 MB), so they are reported as bytes, never as an HBM rate
                     "scene_bytes_per_launch_cache_served": int(scene_b / launches),
                     "total_ms": round(ms, 3)}
        if kc.get("dram_bytes_per_launch") and stream_b:
            res[name]["traffic_over_algorithmic"] = round(kc["dram_bytes_per_launch"] / (stream_b / launches), 2)
            if kc.get("dram_bytes_per_launch_raw"):  # [FETCH_SIZE x1, x2] + WRITE_SIZE over the algorithmic bytes
                res[name]["traffic_over_algorithmic_range"] = [
                    round(kc["dram_bytes_per_launch_raw"] / (stream_b / launches), 2),
                    res[name]["traffic_over_algorithmic"]]
        if kc.get("valu_insts_per_launch"):
            g = kc["valu_insts_per_launch"] / avg_s / 1e9
            res[name]["valu"] = {"achieved": round(g, 1), "peak": VALU_PEAK_GINST, "unit": "G wave-instr/s",
                                 "frac": round(g / VALU_PEAK_GINST, 4),
                                 "insts_per_launch": int(kc["valu_insts_per_launch"])}
    if fallback:
        res[shadow_kernel] = fallback
    return res


def single_lane_pass(cfg, world, rank, spp_per_step, steps):
    """Per-kernel launch times with ONE batch in flight (RTMI_LANES=1): with two lanes a launch's HIP-event time
    also covers the other lane's kernels sharing the CUs, so per-kernel rooflines come from this pass (the rocprof
    kernel traces under profiles/ are single-lane too).  Untimed for `value`; same workload and step size."""
    old = {k: os.environ.get(k) for k in ("RTMI_LANES", "RTMI_NO_STAGE_EVENTS")}
    os.environ["RTMI_LANES"] = "1"
    os.environ.pop("RTMI_NO_STAGE_EVENTS", None)  # this pass times every stage
    try:
        r1 = Renderer(cfg, device=torch.cuda.current_device())
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    r1.set_shard(32, world, rank)
    W, H = cfg.film.res
    film = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    spp = cfg.sampler.spp()
    n = spp_per_step * world
    i0 = 0

    def step():
        nonlocal i0
        if i0 + n > spp:
            i0 = 0
        r1.render_pass_device(i0, i0 + n, film.data_ptr(), stream.cuda_stream)
        i0 += n

    step()
    torch.cuda.synchronize()
    r1.reset_stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = r1.stats()
    del r1
    return st, dt


def effective_cpus(cgroup_root="/sys/fs/cgroup", affinity=None):
    """CPUs this process may actually use: the affinity mask, capped by the cgroup CPU quota (cgroup v2 cpu.max or v1
    cfs_quota_us / cfs_period_us).  os.cpu_count() reports the whole machine (256 on the GPU boxes) although a
    one-GPU box's container gets a share of it."""
    aff = affinity
    if aff is None:
        try:
            aff = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            aff = os.cpu_count() or 1
    quota, src = None, "none"
    root = Path(cgroup_root)
    try:
        q, per = (root / "cpu.max").read_text().split()[:2]
        src = f"cgroup v2 cpu.max = {q} {per}"
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            q = int((root / "cpu" / "cpu.cfs_quota_us").read_text())
            per = int((root / "cpu" / "cpu.cfs_period_us").read_text())
            src = f"cgroup v1 cfs_quota_us = {q}, cfs_period_us = {per}"
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    eff = aff if quota is None else max(1, min(aff, int(quota)))
    return eff, {"affinity_cpus": aff, "nproc": os.cpu_count(), "cgroup_quota_cpus": quota, "cgroup": src}


def project_shards(r, cfg, n, spp_per_step, steps, warmup, stream):
    """Tile-parallel efficiency at n GPUs projected from one GPU (RayTracerTestApp.h:372-397 is the
    dispatch this replaces): rank k of an n-GPU run renders shard k of rt_set_shard(32, n, k) — every n-th 32x32
    tile — for spp_per_step * n sample indices per step (weak scaling: the same samples per GPU as the 1-GPU step).
    Each shard is rendered here alone, for the same number of steps; a step of the n-GPU run lasts as long as its
    slowest shard, so the efficiency is mean / max of the per-shard step times; `efficiency_with_reduce` also charges
    the once-per-frame film reduce (33 MB at 1080p: a measured on-device copy plus the modelled xGMI transfer,
    frame_reduce_cost) to the steps of the frame."""
    W, H = cfg.film.res
    film = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    per, spp = spp_per_step * n, cfg.sampler.spp()
    rows = []
    for k in range(n):
        r.set_shard(32, n, k)
        i0 = 0

        def step():
            nonlocal i0
            if i0 + per > spp:
                i0 = 0
            r.render_pass_device(i0, min(spp, i0 + per), film.data_ptr(), stream.cuda_stream)
            i0 += per

        for _ in range(max(1, warmup)):
            step()
        torch.cuda.synchronize()
        r.reset_stats()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        rows.append({"shard": k, "ms_per_step": round(dt * 1e3, 3), "samples_per_step": int(r.stats()["samples"] / steps)})
    ms = [x["ms_per_step"] for x in rows]
    eff = sum(ms) / len(ms) / max(ms)
    red = frame_reduce_cost(film, n, per, spp)
    step_red = max(ms) + red["per_step_ms"]
    return {"n": n, "efficiency": round(eff, 4), "max_ms": max(ms),
            "mean_ms": round(sum(ms) / len(ms), 3), "shards": rows,
            "efficiency_with_reduce": round(sum(ms) / len(ms) / step_red, 4), "frame_reduce": red,
            "basis": f"each shard of rt_set_shard(32, {n}, k) alone on this GPU, {per} indices per step "
                     f"({steps} steps after {max(1, warmup)} warmup): mean / max step time; with_reduce adds the "
                     f"once-per-frame film reduce (frame_reduce) spread over the frame's steps to the slowest step"}


def frame_reduce_cost(film, n, per, spp, link_gbs=153.0, reps=20):
    """The once-per-frame film reduce of an n-GPU run (distributed.FrameLoop: torch.distributed.reduce(SUM) onto rank
    0), costed per step.  Measured here: a device-to-device copy of the whole film on this GPU (the copy every rank's
    film makes on its way through RCCL's buffers; 33 MB at 1080p).  Modelled: the xGMI transfer of a ring reduce,
    2 (n - 1) / n film sizes over one link at link_gbs (MI355X_MICROARCH: 7 links x ~153 GB/s per GPU; RCCL's ring
    reduce moves that much per link).  The frame is spp indices, a step renders per = spp_per_step x n of them."""
    dst = torch.empty_like(film)
    for _ in range(2):
        dst.copy_(film)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(film)
    e1.record()
    torch.cuda.synchronize()
    copy_ms = e0.elapsed_time(e1) / reps
    nbytes = film.numel() * film.element_size()
    xgmi_ms = 2 * (n - 1) / n * nbytes / (link_gbs * 1e9) * 1e3
    steps_per_frame = max(1.0, spp / per)
    per_frame = copy_ms + xgmi_ms
    return {"film_bytes": nbytes, "d2d_copy_ms_measured": round(copy_ms, 4), "xgmi_ring_reduce_ms_model": round(xgmi_ms, 4),
            "per_frame_ms": round(per_frame, 4), "steps_per_frame": round(steps_per_frame, 3),
            "per_step_ms": round(per_frame / steps_per_frame, 4)}


def cpu_baseline(cfg, seconds):
    """Oracle (C++ restatement, `port`) on the host threads this process may use, as RayTracerTestApp.h:372-397
    spawns hardware_concurrency() threads; built -O3 -march=native on this host; bounded sample: a
    horizontal band of full rows of the same frame, sized per thread count to a share of `seconds` of wall time.
    A thread sweep (1, 8, the effective CPU count E, 2E) shows where the host saturates; `value` and `cores` are the
    E-thread point (E = the affinity mask capped by the cgroup CPU quota, effective_cpus)."""
    from oracle import oracle
    oracle.use_native()
    o = oracle.OracleScene(cfg)
    W, H = cfg.film.res
    spp = cfg.sampler.spp()
    eff, cpuinfo = effective_cpus()

    def run(threads, budget):
        # a band of full rows at sample index 0, grown to the whole frame, then more sample indices of the frame
        rows, nidx = max(1, min(H, threads)), 1
        while True:
            y0 = H // 2 - rows // 2
            pix = np.arange(y0 * W, (y0 + rows) * W, dtype=np.int32)
            t0 = time.perf_counter()
            o.render(0, nidx, nthreads=threads, pixel_ids=pix)
            dt = time.perf_counter() - t0
            if dt > budget * 0.5 or nidx >= spp:
                return len(pix) * nidx / dt / 1e6, len(pix) * nidx, dt, nidx
            grow = max(2.0, budget / max(dt, 1e-3))
            if rows < H:
                rows = min(H, int(rows * grow))
            else:
                nidx = min(spp, int(np.ceil(nidx * grow)))

    points = sorted({1, min(8, eff), eff, min(2 * eff, 512)})
    share = {t: (0.5 if t == eff else 0.15) for t in points}
    sweep, main = [], None
    for t in points:
        v, n, dt, k = run(t, seconds * share[t])
        sweep.append({"threads": t, "msamples_s": round(v, 4), "samples": n, "seconds": round(dt, 2)})
        if t == eff:
            main = (v, n, dt, k)
    v1 = sweep[0]["msamples_s"]
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    v, n, dt, k = main
    return {"value": round(v, 4), "unit": "Msamples/s", "cores": eff, "kind": "port",
            "effective_cpus": eff, **cpuinfo, "thread_sweep": sweep,
            "speedup_at_cores": round(v / v1, 2) if v1 else None,
            "single_thread": v1, "cpu_model": model,
            "build": "g++ -O3 -march=native -ffp-contract=off (built on this host)",
            "sample": f"oracle C++ restatement (same octree BFS, watertight test, path integrator): {n} samples = "
                      f"{n // W // k} full rows of the {W}x{H} frame x sample indices 0..{k - 1} on {eff} threads "
                      f"(affinity capped by the cgroup quota), {dt:.1f} s"}


def main():
    a = parse()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(local if world > 1 else 0)
    # RCCL over xGMI; a finite collective timeout + async error handling: a dead rank fails the run, not hangs it
    world, rank = init_distributed("nccl", device_id=torch.device("cuda", local) if world > 1 else None)
    W, H = (int(x) for x in a.res.split("x"))
    if a.config == "cornell":
        cfg = scene.cfg_cornell(res=(W, H), spp_side=16, max_depth=5)
        workload = (f"BASELINE configs[1]: Cornell box {W}x{H} @ 256 spp (16x16 stratified jittered), "
                    f"diffuse + NEE, max depth 5, 1 quad light, 36 triangles")
    elif a.config == "cfg4":
        cfg = scene.cfg4_mixed(res=(W, H))
        workload = (f"BASELINE configs[3]: mixed scene {W}x{H} @ 1024 spp: 98k-tri mesh + diffuse/mirror/BK7-glass "
                    f"spheres, quad + disk + point + sun lights, NEE + MIS, max depth 5")
    elif a.config == "cfg5":
        W, H = (3840, 2160) if a.res == "1920x1080" else (W, H)
        cfg = scene.cfg5_spectral(res=(W, H))
        workload = (f"BASELINE configs[4]: spectral (8 hero wavelengths) mixed scene {W}x{H} @ 2048 spp, NEE + MIS")
    else:
        cfg = scene.cfg3_blob(res=(W, H), spp_side=16, max_depth=5)
        cfg.sampler = scene.StratifiedSampler(32, 16, True, 0)  # 512 spp
        workload = (f"BASELINE configs[2]: 98k-triangle procedural mesh in the Cornell box {W}x{H} @ 512 spp "
                    f"(32x16 stratified jittered), diffuse + NEE, max depth 5, 1 quad light")
    spp = cfg.sampler.spp()
    r = Renderer(cfg, device=torch.cuda.current_device())
    r.set_shard(32, world, rank)
    film = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    # progressive frames: `spp_per_step * world` indices per step, one RCCL reduce per completed frame
    loop = FrameLoop(spp, a.spp_per_step * world, film, dst=0)

    def step():
        return loop.step(lambda i0, i1, f: r.render_pass_device(i0, i1, f.data_ptr(), stream.cuda_stream))

    tm = timed_steps(step, a.steps, a.warmup, torch.cuda.synchronize, lambda: r.stats()["samples"], r.reset_stats)
    dt, total_samples = tm["dt"], tm["total"]
    st = r.stats()
    value = total_samples / dt / 1e6
    # roofline of the dominant kernel (most HIP-event time), from a single-lane pass (see single_lane_pass)
    # PMC bytes / VALU instructions (profiles/counters_<config>.json, tools/counters.py) are only valid for the
    # workload AND the library build they measured: they are used only when their build id is the loaded library's
    counters, cstat = None, None
    cf = COUNTERS_DIR / f"counters_{a.config}.json"
    loaded = capi.library_sha16()
    if cf.exists():
        cj = json.loads(cf.read_text())
        cstat = {"file": str(cf.relative_to(ROOT)), "tag": cj.get("tag"), "lib_sha16": cj.get("lib_sha16"),
                 "loaded_lib_sha16": loaded}
        if cj.get("lib_sha16") == loaded:
            counters = cj.get("kernels")
            cstat["status"] = "current build"
        else:
            cstat["status"] = "stale (another build): traffic / valu omitted"
    else:
        cstat = {"status": "none: traffic / valu omitted", "loaded_lib_sha16": loaded}
    roofline, st1 = {}, None
    if rank == 0 and not a.no_single_lane:
        st1, dt1 = single_lane_pass(cfg, world, rank, a.spp_per_step, a.steps)
        # multi-level scenes sort their bounce rays unless RTMI_SORT=0 (decided by the configuration, not by whether
        # the sort's stage events recorded time)
        sorted_b = a.config != "cornell" and os.environ.get("RTMI_SORT", "1") not in ("0", "")
        rl = kernel_rooflines(st1, counters, "k_path_nee" if a.config in ("cfg4", "cfg5") else "k_path_shadow",
                              sorted_bounces=sorted_b,
                              n_lights=len(cfg.model.lights))
        dom = max(rl, key=lambda k: rl[k]["total_ms"])
        roofline = dict(rl[dom])
        roofline["basis"] = (f"single-lane pass (RTMI_LANES=1, {a.steps} steps, {dt1 / a.steps * 1e3:.3f} ms/step): "
                             f"{roofline['launches'] / a.steps:g} launches per step x {roofline['avg_launch_ms']} ms")
        roofline["ms_per_step_single_lane"] = round(dt1 / a.steps * 1e3, 3)
        roofline["limiter"] = "VALU issue and memory latency (box + watertight triangle tests); see DESIGN.md §4"
        roofline["other_kernels"] = {k: v for k, v in rl.items() if k != dom}
        roofline["counters"] = cstat
    # Two batches run concurrently on two streams in the timed region (DESIGN.md §4 lanes); the node-level figure
    # divides every kernel's §8(d) stream bytes (generate 96 B/sample, trace 40 B/ray, shade 312 B/bounce + 32 B per
    # shadow ray, film 128 B/sample) by the wall time of the timed region.
    node_b = 96 * st["samples"] + (40 + 312) * st["rays"] + 32 * st["shadow_rays"] + 128 * st["samples"]
    node_a = node_b / dt / 1e9
    roofline["node"] = {"achieved": round(node_a, 1), "frac": round(node_a / HBM_PEAK_GBS, 4),
                        "bytes_per_step": int(node_b / a.steps), "lanes": int(os.environ.get("RTMI_LANES", "2")),
                        "basis": "all kernels' algorithmic stream bytes / wall time of the timed region"}
    out = {
        "metric": "Msamples/s (whole node) at 1920x1080; achieved HBM GB/s vs roofline",
        "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "ranks": tm["ranks"],
        "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (procedural Cornell box scene, no datasets)",
        "config": {"workload": workload,
                   "res": [W, H], "spp_total": spp, "spp_per_step_per_gpu": a.spp_per_step, "max_depth": 5,
                   "parallelism": f"pixel-tile shards x{world} (32x32 tiles) + RCCL film reduce"},
        "roofline": roofline,
        # per-stage GPU time per step from the single-lane pass (HIP events around each stage on the one stream: they
        # sum to at most that pass's ms_per_step); the two-lane timed region overlaps the lanes' stages, so its
        # event spans include the other lane's kernels and are not per-stage times
        "stage_ms": ({k: round(st1[k] / a.steps, 3) for k in ("ms_generate", "ms_sort", "ms_trace", "ms_shade",
                                                               "ms_shadow", "ms_film")} | {
            "basis": "single-lane pass, ms per step (sum <= roofline.ms_per_step_single_lane)"} if st1 else None),
        "counters": {k: st[k] for k in ("samples", "rays", "shadow_rays", "nodes_tested", "tris_tested",
                                        "shadow_nodes_tested", "shadow_tris_tested", "hits", "fallback_rays",
                                        "shadow_fallback_rays")},
    }
    if world == 1 and a.project_shards > 1:
        pj = project_shards(r, cfg, a.project_shards, a.spp_per_step, a.steps, a.warmup, stream)
        out[f"projected_tile_efficiency_{a.project_shards}"] = pj["efficiency"]
        out[f"projected_tile_efficiency_{a.project_shards}_with_reduce"] = pj["efficiency_with_reduce"]
        out["shard_projection"] = pj
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, a.cpu_seconds)
        out["gpu_over_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
