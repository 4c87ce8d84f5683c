#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the oracle (the CPU restatement).

The reference ships no golden data; these fixtures pin the oracle against regression and
give the GPU suite an on-disk target.  Each fixture stores the inputs' identity (config parameters + a
SHA-256 of the mesh arrays) and the expected outputs.  Re-run only when a deliberate semantic change is
made, and say so in the commit.
"""
import hashlib
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

from computational_ray_tracer_amd import scene  # noqa: E402
from oracle.oracle import OracleScene  # noqa: E402


def mesh_hash(model):
    h = hashlib.sha256()
    for a in (model.positions, model.normals, model.indices):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def cfg0_small():
    return scene.cfg0_reference(res=(96, 96), frequency=16, n_index=11)


def cornell_small():
    return scene.cfg_cornell(res=(48, 48), spp_side=4)


def sample_pairs(n=512, npx=96 * 96, nidx=11, seed=11):
    rng = np.random.default_rng(seed)
    return rng.integers(0, npx, n).astype(np.int32), rng.integers(0, nidx, n).astype(np.int32)


def main():
    from computational_ray_tracer_amd.renderer import records_to_arrays
    cfg = cfg0_small()
    o = OracleScene(cfg)
    pix, idx = sample_pairs()
    rec = records_to_arrays(o.samples(pix, idx))
    film = o.render(0, 11)
    oc = o.octree()
    np.savez_compressed(HERE / "cfg0_96.npz", mesh_sha256=mesh_hash(cfg.model), pixel_ids=pix, indices=idx,
                        **{f"rec_{k}": v for k, v in rec.items()}, film=film,
                        oct_bounds=oc["bounds"], oct_child=oc["child"], oct_leaf_count=oc["leaf_count"],
                        oct_refs=oc["refs"], backface=o.backface_flags())
    cc = cornell_small()
    oc2 = OracleScene(cc)
    f2 = oc2.render(0, 16)
    np.savez_compressed(HERE / "cornell_48.npz", mesh_sha256=mesh_hash(cc.model), film=f2, resolved=oc2.resolve(f2))
    print("wrote", sorted(p.name for p in HERE.glob("*.npz")))


if __name__ == "__main__":
    main()
