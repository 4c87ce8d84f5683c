#!/usr/bin/env python3
"""Treelet-queue cost model for the multi-level closest-hit walk.

Builds CFG3's closest-hit BVH exactly as the upload does (rt_debug_bvh_build, no GPU), makes N bounce rays — origins
area-uniform on the scene's triangles, offset along the normal, cosine-distributed directions (outward from the mesh,
into the room from the walls) — orders them by the product's coherence-sort key (origin-major, 3 direction / 3 origin
bits: rt_internal.h ray_sort_key), and runs tools/treelet_sim.cpp on them for several treelet budgets.

  python3 tools/treelet_sim.py [n_rays] > profiles/r06_treelet_model.txt
"""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from computational_ray_tracer_amd import scene  # noqa: E402
from computational_ray_tracer_amd.renderer import build_bvh_host  # noqa: E402
from test_canonical_traversal import _unit, _world_tris  # noqa: E402


def spread3(v):
    v = v.astype(np.uint32) & 0x1FF
    v = (v | (v << 16)) & 0x030000FF
    v = (v | (v << 8)) & 0x0300F00F
    v = (v | (v << 4)) & 0x030C30C3
    v = (v | (v << 2)) & 0x09249249
    return v


def sort_key(o, d, lo, scale, dir_bits=3, org_bits=3):
    """rt_internal.h ray_sort_key, origin-major (the simple path's key)."""
    oct_ = (d[:, 0] < 0) * 4 + (d[:, 1] < 0) * 2 + (d[:, 2] < 0)
    s = np.abs(d).sum(1)
    G = float(1 << dir_bits)
    ux = np.minimum(np.abs(d[:, 0]) / s * G, G - 1).astype(np.uint32)
    uy = np.minimum(np.abs(d[:, 1]) / s * G, G - 1).astype(np.uint32)
    q = np.clip((o - lo) * scale, 0, 511).astype(np.uint32) >> (9 - org_bits)
    mo = (spread3(q[:, 0]) << 2) | (spread3(q[:, 1]) << 1) | spread3(q[:, 2])
    dk = (oct_.astype(np.uint32) << (2 * dir_bits)) | (ux << dir_bits) | uy
    return (mo << (3 + 2 * dir_bits)) | dk


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    cfg = scene.cfg3_blob(res=(64, 36), spp_side=2)
    b = build_bvh_host(cfg.model, 0)
    tris = _world_tris(cfg.model)
    rng = np.random.default_rng(3)
    area = 0.5 * np.linalg.norm(np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0]), axis=1)
    pick = rng.choice(len(tris), n, p=area / area.sum())
    u, v = rng.uniform(size=(2, n))
    sw = u + v > 1
    u[sw], v[sw] = 1 - u[sw], 1 - v[sw]
    t = tris[pick]
    p = t[:, 0] + u[:, None] * (t[:, 1] - t[:, 0]) + v[:, None] * (t[:, 2] - t[:, 0])
    ng = _unit(np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0]))
    n_room = len(tris) - 98_000                      # the Cornell walls and light come first (scene.cornell_box)
    mesh = pick >= n_room
    ref = np.where(mesh[:, None], tris[n_room:].reshape(-1, 3).mean(0), np.array([278.0, 273.0, 280.0]))
    face = np.sum(ng * (p - ref), 1) * np.where(mesh, 1.0, -1.0) > 0   # outward on the mesh, inward on the walls
    ng = np.where(face[:, None], ng, -ng)
    a1 = _unit(np.cross(ng, np.where(np.abs(ng[:, :1]) > 0.9, [[0.0, 1.0, 0.0]], [[1.0, 0.0, 0.0]])))
    a2 = np.cross(ng, a1)
    r1, r2 = rng.uniform(size=(2, n))
    rr, ph = np.sqrt(r1), 2 * np.pi * r2
    d = _unit(a1 * (rr * np.cos(ph))[:, None] + a2 * (rr * np.sin(ph))[:, None] + ng * np.sqrt(1 - r1)[:, None])
    o = p + ng * (1e-4 * (1 + np.abs(p).max(1)))[:, None]
    lo = tris.reshape(-1, 3).min(0)
    scale = 512.0 / (tris.reshape(-1, 3).max(0) - lo)
    key = sort_key(o, d, lo, scale)
    order = np.argsort(key, kind="stable")
    rays = np.c_[o, d][order].astype(np.float32)
    exe = ROOT / "tools" / "_build" / "treelet_sim"
    exe.parent.mkdir(exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), str(ROOT / "tools" / "treelet_sim.cpp")], check=True)
    with tempfile.TemporaryDirectory() as td:
        fn, ft, fr = (os.path.join(td, x) for x in ("n.f32", "t.f32", "r.f32"))
        b["nodes"].astype(np.float32).tofile(fn)
        b["tiles"].astype(np.float32).tofile(ft)
        rays.tofile(fr)
        print(f"# CFG3 closest-hit BVH (rt_debug_bvh_build), {n} cosine bounce rays in coherence-sort order "
              f"(mesh {mesh.mean():.2f} of the origins)", flush=True)
        subprocess.run([str(exe), fn, str(len(b["nodes"])), ft, str(len(b["tiles"])), fr, str(n), str(float(b["consts"][0])),
                        "8192", "16384", "24576", "32768", "65536"], check=True)


if __name__ == "__main__":
    main()
