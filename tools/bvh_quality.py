#!/usr/bin/env python3
"""BVH quality on the CPU: node visits, child-box tests and triangle tests per ray of the restated device walk
(oracle Bvh8) over the BVH the product builds (rt_debug_bvh_build, so RTMI_BVH_CI / RTMI_BVH_LEAF / RTMI_BVH_ANY
apply), for the bounce and shadow rays of a path-traced frame of CFG3 / CFG4's mesh (camera rays, their hits, a
diffuse bounce and a shadow ray to the ceiling light from each hit, as tests/test_canonical_traversal.py builds them).

usage: python tools/bvh_quality.py [cfg3|cfg4] [n_rays]     (prints one JSON line)
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from computational_ray_tracer_amd import scene  # noqa: E402
from computational_ray_tracer_amd.renderer import build_bvh_host  # noqa: E402
from oracle import oracle  # noqa: E402
from test_canonical_traversal import _rays, _secondary, _world_tris  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 400_000
    oracle.build()
    cfg = scene.cfg3_blob(res=(64, 36), spp_side=2) if which == "cfg3" else scene.cfg4_mixed(res=(64, 36), spp=(2, 2))
    o = oracle.OracleScene(cfg)
    t0 = time.time()
    bvh, bany = build_bvh_host(cfg.model, 0), build_bvh_host(cfg.model, 2)
    tb = time.time() - t0
    tris = _world_tris(cfg.model)
    light = cfg.model.lights[0]
    rng = np.random.default_rng(7)
    ro, rd = _rays(rng, n, light, tris)
    k = n // 3
    ro, rd = ro[:k], rd[:k]  # the camera-like family
    prim, bt, _ = o.trace(ro, rd, False)
    po, wi, ws, smax = _secondary(rng, ro, rd, prim, bt, tris, light)
    big = np.full(len(po), 1e30, np.float32)
    sb = o.bvh_check(bvh, po, wi, big, bvh_any=bany)  # bounce rays: closest hit (any-hit over the whole segment)
    ss = o.bvh_check(bvh, po, ws, smax, bvh_any=bany)  # shadow rays: any hit to the light
    r = sb["rays"]
    out = {"config": which, "bvh_nodes": len(bvh["nodes"]), "any_nodes": len(bany["nodes"]), "build_s": round(tb, 2),
           "bounce_rays": r,
           "closest_nodes": round(sb["closest_nodes"] / r, 3), "closest_boxes": round(sb["closest_boxes"] / r, 3),
           "closest_tris": round(sb["closest_tris"] / r, 3),
           "shadow_nodes": round(ss["anyhit_nodes"] / r, 3), "shadow_boxes": round(ss["anyhit_boxes"] / r, 3),
           "shadow_tris": round(ss["anyhit_tris"] / r, 3),
           "mismatch": sb["closest_mismatch"] + ss["anyhit_mismatch"],
           "closest_ambiguous": sb["closest_ambiguous"], "shadow_ambiguous": ss["anyhit_ambiguous"],
           "stack_overflows": sb["stack_overflows"] + ss["stack_overflows"], "max_stack": max(sb["max_stack"], ss["max_stack"]),
           "env": {k: v for k, v in os.environ.items() if k.startswith("RTMI_BVH")}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
