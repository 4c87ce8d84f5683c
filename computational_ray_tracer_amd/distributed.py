"""Multi-GPU path: pixel-tile sharding + one film reduce.

Every camera sample is independent given (pixel, index, dimension, seed), so pixels shard with no exchange
during rendering: rank r owns the 32x32 tiles t with t % world == r (interleaved for load balance) and
accumulates its pixels' samples in the reference's per-pixel index order.  The only collective is one
reduce of the full-frame {r,g,b,w} films to rank 0 (RCCL over xGMI on MI355X; gloo on CPU in tests).
Each pixel has exactly one non-zero contributor, so the reduced film is bit-identical to a 1-GPU render.
"""
import os
import time
from datetime import timedelta

import numpy as np


def shard_pixels(res, tile, n_shards, shard_id):
    """Pixel ids owned by `shard_id`, in the work order the library uses (rt_set_shard / build_work in
    csrc/rt_host.cpp): tiles in row-major tile order, 8x8 micro-tiles inside a tile, row-major inside."""
    W, H = res
    tx, ty = -(-W // tile), -(-H // tile)
    out = []
    for t in range(tx * ty):
        if t % n_shards != shard_id:
            continue
        x0, y0 = (t % tx) * tile, (t // tx) * tile
        for my in range(0, tile, 8):
            for mx in range(0, tile, 8):
                ys = np.arange(y0 + my, y0 + my + 8)[:, None]
                xs = np.arange(x0 + mx, x0 + mx + 8)[None, :]
                ok = (ys < H) & (xs < W) & (ys - y0 < tile) & (xs - x0 < tile)
                ids = (ys * W + xs)[ok]
                out.append(ids.reshape(-1))
    return np.concatenate(out).astype(np.int32) if out else np.zeros(0, np.int32)


class FrameLoop:
    """Progressive rendering of whole frames in steps of `per_step` sample indices (RayTracerTestApp.h:347-452
    renders one index per pass over all pixels and resolves the film after each pass).

    Each rank accumulates its own pixels into `film` (device-resident).  When a step completes the frame
    (index `spp` reached) the per-rank films are reduced onto `dst` ONCE — the frame's only collective — the
    completed frame is kept in `frame` on `dst`, and `film` is zeroed so the next frame starts from nothing.
    Reducing only at frame end keeps the collective off the per-step path and never re-adds a rank's
    earlier contributions (an in-place reduce per step would count the root's already-reduced pixels again).

    Aliasing: by default `frame` is one of two buffers that alternate with `film` on dst (no 33 MB copy per frame,
    bench.py), so the tensor `frame` refers to is zeroed and re-used as the accumulation film when the NEXT frame
    starts, and overwritten when the frame after it completes.  A caller that keeps completed frames beyond one
    frame period (saving or displaying them asynchronously) passes keep_frames=True: every completed frame is then
    a fresh tensor the loop never touches again (one device copy per frame).  Ranks other than dst keep no frame.
    """

    def __init__(self, spp, per_step, film, dst=0, keep_frames=False):
        self.spp, self.per_step, self.film, self.dst = int(spp), int(per_step), film, dst
        self.keep_frames = bool(keep_frames)
        self.cursor = 0
        self.frame = None      # last completed (reduced) frame, on dst (see "Aliasing")
        self.frames_done = 0

    def step(self, render):
        """render(i0, i1, film) accumulates indices [i0, i1) of this rank's pixels; returns i1 - i0.

        At frame end only `dst` keeps the reduced frame, by swapping buffers (no copy): the reduced film becomes
        `frame` and the previous frame's buffer, zeroed, the next accumulation film.  The other ranks' films hold
        only their own pixels after the reduce and are simply zeroed."""
        i0 = self.cursor
        i1 = min(self.spp, i0 + self.per_step)
        render(i0, i1, self.film)
        if i1 >= self.spp:
            reduce_film(self.film, dst=self.dst)
            if _rank() == self.dst:
                if self.keep_frames:
                    self.frame = self.film.clone()
                else:
                    spare = self.frame
                    self.frame = self.film
                    self.film = spare if spare is not None else self.film.new_zeros(self.film.shape)
            self.film.zero_()
            self.frames_done += 1
            self.cursor = 0
        else:
            self.cursor = i1
        return i1 - i0


def _rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_initialized() else 0


def reduce_film(film, dst=0):
    """Sum the per-rank films onto `dst` (torch.distributed; backend nccl = RCCL on ROCm, or gloo).  The collective
    is issued whenever a process group exists, at world size 1 too (tests/test_gpu_configs.py runs RCCL that way on
    the one-GPU box); without a group the film is already the whole frame."""
    import torch.distributed as dist
    if dist.is_initialized():
        dist.reduce(film, dst=dst, op=dist.ReduceOp.SUM)
    return film


def init_distributed(backend="nccl", timeout_s=None, device_id=None, force=False):
    """One process per GPU (torchrun's RANK / WORLD_SIZE / MASTER_* environment).  Every collective gets a finite
    timeout (RTMI_DIST_TIMEOUT seconds, default 300) and, on RCCL, asynchronous error handling that tears the process
    down, so a rank that dies or hangs makes the others fail with a non-zero exit instead of waiting forever.
    At world size 1 no group is created unless `force` (the world-1 RCCL test).  Returns (world, rank)."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if (world > 1 or force) and not dist.is_initialized():
        if timeout_s is None:
            timeout_s = float(os.environ.get("RTMI_DIST_TIMEOUT", "300"))
        if backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        kw = {"timeout": timedelta(seconds=timeout_s)}
        if device_id is not None:
            kw["device_id"] = device_id
        dist.init_process_group(backend, **kw)
    return world, rank


def timed_steps(step, steps, warmup, sync, samples, reset=None):
    """bench.py's timed region, shared with the multi-process CPU tests: `warmup` untimed steps, then exactly `steps`
    steps bracketed by barrier + `sync()` on both sides; the wall time is the MAX over ranks and the per-rank sample
    counts (`samples()` after the timed steps, `reset()` before them) are gathered to every rank.
    Returns dict(dt=max seconds, total=samples over all ranks, ranks=[{rank, samples, s}, ...])."""
    import torch
    import torch.distributed as dist
    multi = dist.is_initialized()  # (a world-1 group too: its barrier and all_gather run)
    for _ in range(warmup):
        step()
    sync()
    if reset:
        reset()
    if multi:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if multi:
        dist.barrier()
    dt = time.perf_counter() - t0
    mine = float(samples())
    if not multi:
        return {"dt": dt, "total": mine, "ranks": [{"rank": 0, "samples": int(mine), "s": round(dt, 6)}]}
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    v = torch.tensor([mine, dt], dtype=torch.float64, device=dev)
    allv = [torch.zeros_like(v) for _ in range(dist.get_world_size())]
    dist.all_gather(allv, v)
    ranks = [{"rank": r, "samples": int(x[0].item()), "s": round(float(x[1].item()), 6)} for r, x in enumerate(allv)]
    return {"dt": max(r["s"] for r in ranks), "total": float(sum(r["samples"] for r in ranks)), "ranks": ranks}
