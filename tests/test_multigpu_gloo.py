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
    if rank == 0:
        q.put((film.numpy().copy(), loop.frame.numpy().copy(), acc.numpy().copy(), pix))
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
