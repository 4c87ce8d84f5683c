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
from computational_ray_tracer_amd.distributed import reduce_film, shard_pixels


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
    if rank == 0:
        q.put(film.numpy().copy())
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
    film2 = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    cfg = scene.cfg_cornell(res=(72, 40), spp_side=2)
    film1 = oracle_lib.OracleScene(cfg).render(0, 4)
    assert np.array_equal(film1.view(np.uint32), film2.view(np.uint32))
