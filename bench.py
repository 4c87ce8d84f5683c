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

from computational_ray_tracer_amd import scene  # noqa: E402
from computational_ray_tracer_amd.distributed import FrameLoop  # noqa: E402
from computational_ray_tracer_amd.renderer import Renderer  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
TRAFFIC_FILE = ROOT / "profiles" / "traffic.json"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--spp-per-step", type=int, default=8)
    p.add_argument("--res", type=str, default="1920x1080")
    p.add_argument("--config", choices=["cornell", "cfg3", "cfg4", "cfg5"], default="cornell",
                   help="cornell = BASELINE configs[1] (the metric's workload); cfg3..cfg5 = configs[2..4]")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    return p.parse_args()


def kernel_rooflines(st, traffic):
    """Per-kernel HBM roofline from the HIP-event launch times of the timed region.

    Algorithmic bytes follow SURVEY.md §8(d): the per-ray HBM streams are `achieved` (k_trace_closest: 40 B per
    ray cast; k_path_shade: 312 B per shaded bounce + 32 B per shadow ray); the §8(d) scene terms (32 B per node
    box test + 40 B per triangle test) are reported beside them as `achieved_incl_scene` — on this 36-triangle
    scene they are scalar-cache/L2 hits (the whole octree is 1.8 KB), so folding them into an HBM rate would
    exceed the HBM peak.  `traffic` is the PMC-measured DRAM bytes per launch (profiles/traffic.json)."""
    ks = {
        "k_trace_closest": (st["ms_trace"], st["launches_trace"], 40 * st["rays"],
                            32 * st["nodes_tested"] + 40 * st["tris_tested"]),
        "k_path_shade": (st["ms_shade"], st["launches_shade"], 312 * st["rays"] + 32 * st["shadow_rays"],
                         32 * st["shadow_nodes_tested"] + 40 * st["shadow_tris_tested"]),
    }
    res = {}
    for name, (ms, launches, stream_b, scene_b) in ks.items():
        launches = max(1, launches)
        avg_s = ms / launches * 1e-3
        a = stream_b / launches / avg_s / 1e9
        res[name] = {"bound": "hbm", "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(a / HBM_PEAK_GBS, 4),
                     "traffic": (traffic or {}).get(name, {}).get("dram_bytes_per_launch"),
                     "kernel": name, "launches": launches, "avg_launch_ms": round(avg_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": int(stream_b / launches),
                     "scene_bytes_per_launch": int(scene_b / launches),
                     "achieved_incl_scene": round((stream_b + scene_b) / launches / avg_s / 1e9, 1),
                     "total_ms": round(ms, 3)}
    return res


def cpu_baseline(cfg, seconds):
    """Oracle (C++ restatement, `port`) on every host thread (hardware_concurrency, as RayTracerTestApp.h:372-397
    spawns), built -O3 -march=native on this host; bounded sample: a horizontal band of full rows of
    the same frame, 1 sample index, sized to ~`seconds` of CPU work."""
    from oracle import oracle
    oracle.use_native()
    OracleScene = oracle.OracleScene
    threads = min(os.cpu_count() or 1, 512)  # the pool's per-box task limit is 1024
    o = OracleScene(cfg)
    W, H = cfg.film.res
    spp = cfg.sampler.spp()
    rows, nidx = 8, 1
    while True:
        y0 = H // 2 - rows // 2
        pix = np.arange(y0 * W, (y0 + rows) * W, dtype=np.int32)
        t0 = time.perf_counter()
        o.render(0, nidx, nthreads=threads, pixel_ids=pix)
        dt = time.perf_counter() - t0
        if dt > seconds * 0.5 or (rows >= H and nidx >= spp):
            break
        grow = max(2.0, seconds / max(dt, 1e-3))
        if rows < H:
            rows = min(H, int(rows * grow))
        else:
            nidx = min(spp, int(nidx * grow))
    n = len(pix) * nidx
    ms = n / dt / 1e6
    # single-thread figure: the same band's first rows on one thread, ~1/8 of the budget
    r1 = max(1, min(rows, int(rows / threads / 8)))
    p1 = pix[: r1 * W]
    t0 = time.perf_counter()
    o.render(0, nidx, nthreads=1, pixel_ids=p1)
    dt1 = time.perf_counter() - t0
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"value": round(ms, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "affinity_cpus": affinity,
            "single_thread": round(len(p1) * nidx / dt1 / 1e6, 4), "cpu_model": model,
            "build": "g++ -O3 -march=native -ffp-contract=off (built on this host)",
            "sample": f"oracle C++ restatement (same octree BFS, watertight test, path integrator), {n} samples = "
                      f"{rows} full rows of the {W}x{H} frame x sample indices 0..{nidx - 1}, "
                      f"{threads} threads (os.cpu_count), {dt:.1f} s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
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

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    r.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    idx_done = 0
    for _ in range(a.steps):
        idx_done += step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = r.stats()
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        tot = torch.tensor([st["samples"]], dtype=torch.float64, device="cuda")
        dist.all_reduce(tot)
        total_samples = float(tot.item())
    else:
        total_samples = float(st["samples"])
    value = total_samples / dt / 1e6
    # roofline of the dominant kernel (most HIP-event time in the timed region)
    traffic = None
    if TRAFFIC_FILE.exists():
        tj = json.loads(TRAFFIC_FILE.read_text())
        if tj.get("config", "cornell") == a.config:  # PMC bytes are only valid for the workload they measured
            traffic = tj.get("kernels")
    rl = kernel_rooflines(st, traffic)
    dom = max(rl, key=lambda k: rl[k]["total_ms"])
    roofline = dict(rl[dom])
    roofline["limiter"] = "VALU issue (octree box + watertight triangle tests); see DESIGN.md §Roofline"
    # Two batches run concurrently on two streams (DESIGN.md §4 lanes), so a launch's HIP-event duration includes
    # time it shares the CUs with the other lane's kernels; the node-level figure divides every kernel's §8(d)
    # stream bytes (generate 96 B/sample, trace 40 B/ray, shade 312 B/bounce + 32 B/shadow ray, film 128 B/sample)
    # by the wall time of the timed region.
    node_b = 96 * st["samples"] + (40 + 312) * st["rays"] + 32 * st["shadow_rays"] + 128 * st["samples"]
    node_a = node_b / dt / 1e9
    roofline["node"] = {"achieved": round(node_a, 1), "frac": round(node_a / HBM_PEAK_GBS, 4),
                        "bytes_per_step": int(node_b / a.steps), "lanes": int(os.environ.get("RTMI_LANES", "2")),
                        "basis": "all kernels' algorithmic stream bytes / wall time of the timed region"}
    roofline["other_kernels"] = {k: v for k, v in rl.items() if k != dom}
    out = {
        "metric": "Msamples/s (whole node) at 1920x1080; achieved HBM GB/s vs roofline",
        "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (procedural Cornell box scene, no datasets)",
        "config": {"workload": workload,
                   "res": [W, H], "spp_total": spp, "spp_per_step_per_gpu": a.spp_per_step, "max_depth": 5,
                   "parallelism": f"pixel-tile shards x{world} (32x32 tiles) + RCCL film reduce"},
        "roofline": roofline,
        "stage_ms": {k: round(st[k], 2) for k in ("ms_generate", "ms_trace", "ms_shade", "ms_shadow", "ms_film")},
        "counters": {k: st[k] for k in ("samples", "rays", "shadow_rays", "nodes_tested", "tris_tested",
                                        "shadow_nodes_tested", "shadow_tris_tested", "hits")},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, a.cpu_seconds)
        out["gpu_over_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
