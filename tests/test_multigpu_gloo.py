"""CPU, world_size 2 over gloo: the N>1 path (tile sharding + one film reduce) reproduces the single-rank
film bit-for-bit.  Each rank renders its shard with the oracle (CPU stand-in for its GPU) and the films are
reduced with torch.distributed exactly as bench.py does with RCCL on MI355X."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from computational_ray_tracer_amd import scene
from computational_ray_tracer_amd.distributed import FrameLoop, reduce_film, shard_pixels


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import OracleScene
    cfg = scene.cfg_cornell(res=(72, 40), spp_side=2)
    o = OracleScene(cfg)
    pix = shard_pixels(cfg.film.res, 16, world, rank)
    film = torch.from_numpy(o.render(0, 4, nthreads=2, pixel_ids=pix))
    reduce_film(film, dst=0)
    # bench.py's progressive frame loop: 2 indices per step (1 per rank), reduce once per completed frame, the
    # accumulation film zeroed for the next frame (a 3rd step starts frame 2 without re-adding frame 1)
    acc = torch.zeros_like(film)
    loop = FrameLoop(4, 2, acc, dst=0)
    render = lambda i0, i1, f: f.add_(torch.from_numpy(o.render(i0, i1, nthreads=2, pixel_ids=pix)))  # noqa: E731
    for _ in range(3):
        loop.step(render)
    assert loop.frames_done == 1
    # only dst keeps the reduced frame (its film buffer swapped out, no clone); the others keep no frame copy
    assert (loop.frame is not None) == (rank == 0)
    if rank == 0:
        assert loop.frame.data_ptr() == acc.data_ptr() and loop.film.data_ptr() != acc.data_ptr()
        q.put((film.numpy().copy(), loop.frame.numpy().copy(), loop.film.numpy().copy(), pix))
    dist.barrier()
    dist.destroy_process_group()


def test_shards_partition_the_frame():
    for res, tile, n in (((1920, 1080), 32, 8), ((72, 40), 16, 3), ((500, 500), 32, 2)):
        allp = np.concatenate([shard_pixels(res, tile, n, r) for r in range(n)])
        assert len(allp) == res[0] * res[1]
        assert np.array_equal(np.sort(allp), np.arange(res[0] * res[1]))


def test_gloo_two_ranks_equal_single_rank(oracle_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    film2, frame, acc, pix0 = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    cfg = scene.cfg_cornell(res=(72, 40), spp_side=2)
    film1 = oracle_lib.OracleScene(cfg).render(0, 4)
    assert np.array_equal(film1.view(np.uint32), film2.view(np.uint32))
    # frame loop: the reduced frame is the sum of the two per-step blocks (each rendered from zero and added,
    # as the test's render callback does); the accumulation film holds only frame 2's first step, own pixels
    o = oracle_lib.OracleScene(cfg)
    two = o.render(0, 2) + o.render(2, 4)
    assert np.array_equal(frame.view(np.uint32), two.view(np.uint32))
    part = np.zeros_like(acc)
    part[pix0] = o.render(0, 2)[pix0]
    assert np.array_equal(acc.view(np.uint32), part.view(np.uint32))


def _timed_worker(rank, world, port, q):
    """bench.py's timed region (distributed.timed_steps) on a frame loop spanning more than one frame: 6 steps of 2
    indices (one per rank) over frames of 4, after 1 warmup step -> frames complete at steps 2, 4 and 6."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from computational_ray_tracer_amd.distributed import init_distributed, timed_steps
    w, r = init_distributed("gloo", timeout_s=120)
    assert (w, r) == (world, rank)
    from oracle.oracle import OracleScene
    cfg = scene.cfg_cornell(res=(40, 24), spp_side=2)
    o = OracleScene(cfg)
    pix = shard_pixels(cfg.film.res, 16, world, rank)
    acc = torch.zeros((40 * 24, 4), dtype=torch.float32)
    loop = FrameLoop(4, 2, acc, dst=0)
    done = {"samples": 0}

    def render(i0, i1, f):
        f.add_(torch.from_numpy(o.render(i0, i1, nthreads=2, pixel_ids=pix)))
        done["samples"] += (i1 - i0) * len(pix)

    tm = timed_steps(lambda: loop.step(render), 6, 1, lambda: None, lambda: done["samples"],
                     lambda: done.update(samples=0))
    assert (loop.frame is not None) == (rank == 0)  # dst-only frame
    if rank == 0:
        q.put((tm, loop.frames_done, loop.frame.numpy().copy(), len(pix)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_timed_steps_over_several_frames(oracle_lib):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_timed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    tm, frames, frame, npix0 = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert frames == 3  # warmup (1 step) + 6 timed steps of 2 indices over 4-index frames: frames end at 2, 4, 6
    assert [r["rank"] for r in tm["ranks"]] == [0, 1]
    assert tm["ranks"][0]["samples"] == 6 * 2 * npix0
    assert tm["total"] == 6 * 2 * 40 * 24 and tm["dt"] == max(r["s"] for r in tm["ranks"])
    # the last completed frame (indices 0..3, rendered as two 2-index steps) equals the single-rank render
    cfg = scene.cfg_cornell(res=(40, 24), spp_side=2)
    o = oracle_lib.OracleScene(cfg)
    two = o.render(0, 2) + o.render(2, 4)
    assert np.array_equal(frame.view(np.uint32), two.view(np.uint32))


def _hung_peer_worker(rank, world, port, q):
    """Rank 1 hangs (never reaches the timed region's barrier); rank 0's collectives must time out and raise."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from computational_ray_tracer_amd.distributed import init_distributed, timed_steps
    init_distributed("gloo", timeout_s=5)
    if rank == 1:
        time.sleep(600)
        return
    t0 = time.time()
    try:
        timed_steps(lambda: None, 2, 0, lambda: None, lambda: 0)
        q.put(("no error", time.time() - t0))
    except Exception as e:  # noqa: BLE001 — the test checks that it is raised, whatever torch calls it
        q.put((type(e).__name__, time.time() - t0))


def test_gloo_hung_peer_fails_instead_of_hanging():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_hung_peer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        what, waited = q.get(timeout=120)
    finally:
        for p in ps:
            p.kill()
            p.join(timeout=30)
    assert what != "no error"
    assert waited < 60, waited


def _worker_frames8(rank, world, port, q):
    """bench.py's frame geometry at N = 8: a 256-index frame, 16 indices per GPU per step (per_step = 16 N = 128), so
    the frame loop must reduce exactly once every spp / (spp_per_step N) = 2 steps, and never in between."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from computational_ray_tracer_amd import distributed as D
    calls = []
    real = D.reduce_film

    def counting(film, dst=0):
        calls.append(len(steps_done))
        return real(film, dst=dst)

    D.reduce_film = counting  # FrameLoop.step calls the module's reduce_film
    res, spp, per_gpu = (64, 32), 256, 16
    pix = torch.from_numpy(shard_pixels(res, 16, world, rank).astype(np.int64))
    film = torch.zeros((res[0] * res[1], 4), dtype=torch.float32)
    loop = FrameLoop(spp, per_gpu * world, film, dst=0, keep_frames=(rank == 0))
    steps_done, frames = [], []

    def render(i0, i1, f):  # every owned pixel gains one unit per sample index of the step
        f[pix] += float(i1 - i0)

    for s in range(7):
        loop.step(render)
        steps_done.append(s)
        if rank == 0 and loop.frame is not None and len(frames) < loop.frames_done:
            frames.append(loop.frame)
    D.reduce_film = real
    q.put((rank, calls, loop.frames_done, loop.cursor,
           [f.numpy().copy() for f in frames] if rank == 0 else None))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_eight_ranks_reduce_once_per_frame():
    """N = 8 (gloo): one reduce per completed 256-index frame — at steps 2, 4, 6 of 7 — on every rank, each reduced
    frame holds every pixel exactly once x 256 indices, and with keep_frames the completed frames stay untouched."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_frames8, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(world):
        r, calls, done, cursor, frames = q.get(timeout=300)
        got[r] = (calls, done, cursor, frames)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    steps_per_frame = 256 // (16 * world)
    assert steps_per_frame == 2
    for r in range(world):
        calls, done, cursor, _ = got[r]
        assert calls == [1, 3, 5], (r, calls)  # 0-based step index at which the frame completed
        assert done == 3 and cursor == 128  # the 7th step started frame 4
    frames = got[0][3]
    assert len(frames) == 3
    for f in frames:
        assert np.all(f == 256.0)
