"""Child process of tests/test_gpu_configs.py::test_rccl_world1_frame_loop (not a test module).

Runs bench.py's multi-GPU machinery at world size 1 on the GPU box with RCCL actually called: the process group is
initialised with backend "nccl" (RCCL on ROCm) before any other GPU work, `reduce_film` issues `dist.reduce` (it
does whenever a group exists), and `timed_steps` runs its barrier + all_gather.  The parent set MASTER_ADDR /
MASTER_PORT / RANK / WORLD_SIZE in this process's environment before it started, so nothing here re-executes.
Prints one JSON line with the checks' inputs; the parent asserts on them.
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from computational_ray_tracer_amd import scene  # noqa: E402
from computational_ray_tracer_amd.distributed import FrameLoop, init_distributed, reduce_film, timed_steps  # noqa: E402
from computational_ray_tracer_amd.renderer import Renderer  # noqa: E402


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    world, rank = init_distributed("nccl", device_id=torch.device("cuda", 0), force=True)
    assert dist.is_initialized() and dist.get_backend() == "nccl" and world == 1 and rank == 0
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}

    # 1. a 1080p film (33 MB) through the same call reduce_film makes: a world-1 SUM reduce is the identity
    g = torch.Generator(device="cuda").manual_seed(5)
    big = torch.rand((1920 * 1080, 4), generator=g, device="cuda", dtype=torch.float32)
    ref = big.clone()
    reduce_film(big, dst=0)
    torch.cuda.synchronize()
    out["reduce_bytes"] = big.numel() * 4
    out["reduce_identity"] = bool(torch.equal(big.view(torch.int32), ref.view(torch.int32)))

    # 2. bench.py's progressive frame loop under timed_steps: two whole frames, each reduced through RCCL
    cfg = scene.cfg_cornell(res=(64, 48), spp_side=2, max_depth=5)   # 4 spp per frame
    r = Renderer(cfg, device=0)
    r.set_shard(32, world, rank)
    film = torch.zeros((64 * 48, 4), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    loop = FrameLoop(cfg.sampler.spp(), 2, film, dst=0)

    def step():
        return loop.step(lambda i0, i1, f: r.render_pass_device(i0, i1, f.data_ptr(), stream.cuda_stream))

    tm = timed_steps(step, 4, 0, torch.cuda.synchronize, lambda: r.stats()["samples"], r.reset_stats)
    out["frames_done"] = loop.frames_done
    out["timed_samples"] = tm["total"]
    out["ranks"] = tm["ranks"]
    frame = loop.frame.cpu().numpy()
    direct = Renderer(cfg, device=0).render_pass(0, cfg.sampler.spp())
    out["frame_equals_direct"] = bool(np.array_equal(frame.view(np.uint32), direct.view(np.uint32)))
    out["frame_nonzero"] = bool((frame[:, 3] > 0).all())
    dist.barrier()
    dist.destroy_process_group()
    print("RCCL_WORLD1 " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
