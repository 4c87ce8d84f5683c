"""GPU parity: the HIP path (through the C-ABI) against the oracle on the same inputs.

Bar: bit-exact hit primitive ids, barycentrics, t, rays, wavelengths, per-sample
radiance/RGB and the accumulated film for the reference integrator; bit-exact films for the build-defined
path integrator (same op order on both sides; tolerance 0, stated per test).
"""
import numpy as np
import pytest

from computational_ray_tracer_amd import capi, scene
from computational_ray_tracer_amd.renderer import Renderer, records_to_arrays

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.fixture(scope="module")
def cfg0_small():
    return scene.cfg0_reference(res=(96, 96), frequency=16, n_index=11)


@pytest.fixture(scope="module")
def pair_small(cfg0_small, oracle_lib):
    return Renderer(cfg0_small), oracle_lib.OracleScene(cfg0_small)


def test_octree_matches_oracle(pair_small):
    g, o = pair_small
    a, b = g.octree(), o.octree()
    assert np.array_equal(bits(a["bounds"]), bits(b["bounds"]))
    assert np.array_equal(a["child"], b["child"])
    assert np.array_equal(a["leaf_count"], b["leaf_count"])
    assert np.array_equal(a["refs"], b["refs"])


def _camera_rays(o, n, seed):
    rng = np.random.default_rng(seed)
    pix = rng.integers(0, o.res[0] * o.res[1], n)
    idx = rng.integers(0, 11, n)
    recs = records_to_arrays(o.samples(pix, idx))
    return recs["ro"], recs["rd"]


@pytest.mark.parametrize("use_cull", [True, False])
def test_trace_camera_rays_bitexact(pair_small, use_cull):
    g, o = pair_small
    ro, rd = _camera_rays(o, 20000, 1)
    pg, bg = g.trace(ro, rd, use_cull)
    po, bo, _ = o.trace(ro, rd, use_cull)
    assert (po >= 0).mean() > 0.2
    assert np.array_equal(pg, po)
    assert np.array_equal(bits(bg), bits(bo))


def test_trace_random_rays_bitexact(pair_small):
    g, o = pair_small
    rng = np.random.default_rng(7)
    n = 20000
    # rays from a shell around the mesh towards random points inside its bounds
    ob = o.octree()["bounds"][0]
    c = (ob[:3] + ob[3:]) / 2
    ext = (ob[3:] - ob[:3])
    ro = (c + rng.normal(size=(n, 3)) * ext).astype(np.float32)
    tgt = (c + (rng.random((n, 3)) - 0.5) * ext * 0.8).astype(np.float32)
    d = tgt - ro
    rd = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    # include axis-aligned directions (d[i] == 0 → ±inf slabs, NaN handling in Bounds3::IntersectP)
    rd[:50] = np.eye(3, dtype=np.float32)[np.arange(50) % 3] * np.where(np.arange(50) % 2, 1, -1)[:, None]
    pg, bg = g.trace(ro, rd, False)
    po, bo, _ = o.trace(ro, rd, False)
    assert np.array_equal(pg, po)
    assert np.array_equal(bits(bg), bits(bo))


def test_sample_records_bitexact(pair_small):
    g, o = pair_small
    rng = np.random.default_rng(3)
    pix = rng.integers(0, 96 * 96, 4096)
    idx = rng.integers(0, 11, 4096)
    rg = records_to_arrays(g.samples(pix, idx))
    ro_ = records_to_arrays(o.samples(pix, idx))
    for k in ("lam", "pdf", "ro", "rd", "prim", "b", "L", "rgb", "weight"):
        assert np.array_equal(np.ascontiguousarray(rg[k]).view(np.uint32), np.ascontiguousarray(ro_[k]).view(np.uint32)), k


def test_cfg0_small_film_bitexact(pair_small):
    g, o = pair_small
    fg = g.render_pass(0, 11)
    fo = o.render(0, 11)
    assert np.array_equal(bits(fg), bits(fo))
    # progressive passes accumulate exactly like one batched pass (RayTracerTestApp.h:420-422)
    f2 = g.new_film()
    for i in range(11):
        g.render_pass(i, i + 1, f2)
    assert np.array_equal(bits(f2), bits(fo))


def test_cfg0_full_reference_workload_bitexact(oracle_lib):
    """SURVEY §8(d) CFG0 at full size: 500x500, indices 0..10, ~20k-triangle octree mesh (2.75 M samples)."""
    cfg = scene.cfg0_reference()
    g = Renderer(cfg)
    fg = g.render_pass(0, 11)
    fo = oracle_lib.OracleScene(cfg).render(0, 11)
    assert np.array_equal(bits(fg), bits(fo))
    st = g.stats()
    assert st["samples"] == 500 * 500 * 11


def test_resolve_matches_oracle(pair_small):
    g, o = pair_small
    f = o.render(0, 3)
    assert np.array_equal(g.resolve(f), o.resolve(f))
    assert np.array_equal(g.resolve(f, srgb=True), o.resolve(f, srgb=True))   # pbrt sRGB encoding (color.h:537-557)


def test_cornell_path_film_bitexact(oracle_lib):
    cfg = scene.cfg_cornell(res=(64, 64), spp_side=4)
    g = Renderer(cfg)
    fg = g.render_pass(0, 16)
    fo = oracle_lib.OracleScene(cfg).render(0, 16)
    bad = np.any(bits(fg) != bits(fo), axis=1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ; max |diff| {np.abs(fg - fo).max()}"


@pytest.mark.parametrize("lanes,scene_kind", [(2, "cornell"), (1, "cornell"), (2, "mesh")])
def test_concurrent_batches_film_bitexact(oracle_lib, monkeypatch, lanes, scene_kind):
    """Several batches per pass (RTMI_BATCH_SAMPLES) alternating between the two lane streams, including an odd
    batch count and a ragged last batch: the film chain must keep every pixel's index order (tolerance 0)."""
    monkeypatch.setenv("RTMI_BATCH_SAMPLES", str(48 * 40 * 2))   # 2 indices per batch
    monkeypatch.setenv("RTMI_LANES", str(lanes))
    if scene_kind == "cornell":
        cfg = scene.cfg_cornell(res=(48, 40), spp_side=3)
    else:
        cfg = scene.cfg3_blob(res=(48, 40), spp_side=3, max_depth=3, frequency=20)
    g = Renderer(cfg)
    fg = g.render_pass(0, 7)                                      # batches {0,1} {2,3} {4,5} {6}
    f2 = g.new_film()
    g.render_pass(0, 3, f2)                                       # a pass boundary inside a lane group
    g.render_pass(3, 7, f2)
    fo = oracle_lib.OracleScene(cfg).render(0, 7)
    assert np.array_equal(bits(fg), bits(fo))
    assert np.array_equal(bits(f2), bits(fo))


@pytest.mark.parametrize("dfs", [0, 1])
def test_shadow_queue_film_bitexact(oracle_lib, monkeypatch, dfs):
    """Multi-level octree with the NEE shadow rays queued and traced by k_path_shadow (RTMI_SHADOW_QUEUE=1), BFS
    or depth-first any-hit: every L gets its additions in the same order, so the film is bit-exact (tolerance 0)."""
    monkeypatch.setenv("RTMI_SHADOW_QUEUE", "1")
    monkeypatch.setenv("RTMI_SHADOW_DFS", str(dfs))
    monkeypatch.setenv("RTMI_BATCH_SAMPLES", str(48 * 40 * 2))   # several batches on both lanes
    cfg = scene.cfg3_blob(res=(48, 40), spp_side=3, max_depth=4, frequency=20)
    g = Renderer(cfg)
    fg = g.render_pass(0, 5)
    fo = oracle_lib.OracleScene(cfg).render(0, 5)
    assert np.array_equal(bits(fg), bits(fo))
    st = g.stats()
    assert st["shadow_rays"] > 0 and st["shadow_nodes_tested"] > 0


def test_shards_sum_to_full_film(oracle_lib):
    from computational_ray_tracer_amd.distributed import shard_pixels
    cfg = scene.cfg_cornell(res=(80, 48), spp_side=2)
    full = Renderer(cfg).render_pass(0, 4)
    acc = np.zeros_like(full)
    for sid in range(3):
        r = Renderer(cfg)
        r.set_shard(16, 3, sid)
        part = r.render_pass(0, 4)
        owned = np.zeros(80 * 48, bool)
        owned[shard_pixels((80, 48), 16, 3, sid)] = True
        assert np.array_equal(part[:, 3] > 0, owned)  # the library owns exactly the Python-mirrored tiles
        acc += part
    assert np.array_equal(bits(acc), bits(full))


def test_octree_path_mode_bfs_queue(oracle_lib):
    """Path integrator on a multi-level octree (BFS group queue in use), bit-exact vs the oracle."""
    base = scene.cfg0_reference(res=(48, 48), frequency=16, n_index=4)
    m = base.model
    m.cull_backfaces = False
    m.materials = [(scene.CORNELL_WHITE, 0.0), ((0.0, 0.0, 0.0), 40.0)]
    m.tri_material = np.zeros(len(m.indices), np.int32)
    m.lights = [dict(p=(-150.0, 250.0, 650.0), e1=(300.0, 0.0, 0.0), e2=(0.0, 0.0, 300.0), n=(0.0, -1.0, 0.0),
                     material=1)]
    from computational_ray_tracer_amd import capi
    cfg = scene.Config("mesh_path", m, base.camera, scene.StratifiedSampler(2, 2, True, 0), base.film,
                       scene.Integrator(capi.RT_INTEGRATOR_PATH, max_depth=3), 0, 4)
    g = Renderer(cfg)
    assert g.octree()["max_queue_groups"] > 1
    fg = g.render_pass(0, 4)
    fo = oracle_lib.OracleScene(cfg).render(0, 4)
    assert np.array_equal(bits(fg), bits(fo))


@pytest.fixture(scope="module")
def cfg3_pair(oracle_lib):
    cfg = scene.cfg3_blob(res=(96, 54), spp_side=2, max_depth=5)
    return cfg, Renderer(cfg), oracle_lib.OracleScene(cfg)


def test_cfg3_octree_and_ring(cfg3_pair):
    """CFG3 (98k-triangle mesh in the Cornell box): same octree as the oracle, and a BFS frontier bound
    beyond the compiled private FIFOs, so traversal runs on the HBM ring (qcap 0)."""
    _, g, o = cfg3_pair
    a, b = g.octree(), o.octree()
    assert np.array_equal(bits(a["bounds"]), bits(b["bounds"]))
    assert np.array_equal(a["child"], b["child"])
    assert np.array_equal(a["refs"], b["refs"])
    assert a["max_queue_groups"] > 1024


def test_cfg3_trace_random_rays_bitexact(cfg3_pair):
    _, g, o = cfg3_pair
    rng = np.random.default_rng(11)
    n = 40000
    ro = np.stack([rng.uniform(5, 550, n), rng.uniform(5, 543, n), rng.uniform(5, 554, n)], 1).astype(np.float32)
    d = rng.normal(size=(n, 3))
    tgt = np.array([278.0, 150.0, 280.0]) + rng.normal(size=(n, 3)) * 60  # half of the rays aim at the mesh
    d[: n // 2] = tgt[: n // 2] - ro[: n // 2]
    rd = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    pg, bg = g.trace(ro, rd, False)
    po, bo, _ = o.trace(ro, rd, False)
    assert (po >= 12).mean() > 0.3   # mesh triangles follow the 12 wall/light triangles
    assert np.array_equal(pg, po)
    assert np.array_equal(bits(bg), bits(bo))
    # shadow query (LDS/HBM-ring FIFO traversal with early exit), tmax around the closest hit distance
    t = np.where(po >= 0, bo[:, 3], 400.0)
    tmax = (t * rng.choice([0.5, 0.999, 1.0, 1.001, 2.0], size=n)).astype(np.float32)
    og = g.occluded(ro, rd, tmax)
    assert np.array_equal(og, o.occluded(ro, rd, tmax))
    assert 0.2 < og.mean() < 0.9


def test_cfg3_path_film_bitexact(cfg3_pair):
    cfg, g, o = cfg3_pair
    fg = g.render_pass(0, 4)
    fo = o.render(0, 4)
    bad = np.any(bits(fg) != bits(fo), axis=1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ"


def test_cfg3_lanes_overlap_with_ring_spills(cfg3_pair, oracle_lib, monkeypatch):
    """Two lanes whose trace / shade kernels run concurrently on a scene whose BFS FIFOs spill to the HBM overflow
    ring (qcap 0): each lane has its own ring, so the film is bit-exact (tolerance 0).  Small batches (one index
    each) keep both lanes busy at once across the pass."""
    cfg, _, o = cfg3_pair
    monkeypatch.setenv("RTMI_BATCH_SAMPLES", str(96 * 54))
    monkeypatch.setenv("RTMI_LANES", "2")
    g = Renderer(cfg)
    fg = g.render_pass(0, 4)
    fo = o.render(0, 4)
    bad = np.any(bits(fg) != bits(fo), axis=1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ"


@pytest.fixture(scope="module")
def cfg4_small():
    return scene.cfg4_mixed(res=(96, 54), spp=(2, 2), frequency=16)


def test_cfg4_trace_with_shapes_bitexact(cfg4_small, oracle_lib):
    """Closest hit = octree, then spheres / disk in list order with the running tMax (hit ids n_tris + k)."""
    g, o = Renderer(cfg4_small), oracle_lib.OracleScene(cfg4_small)
    rng = np.random.default_rng(5)
    n = 30000
    ro = np.stack([rng.uniform(5, 550, n), rng.uniform(5, 543, n), rng.uniform(5, 554, n)], 1).astype(np.float32)
    centres = np.array([[120, 60, 330], [430, 70, 120], [215, 65, 140], [150, 540, 430]], float)
    tgt = centres[rng.integers(0, 4, n)] + rng.normal(size=(n, 3)) * 30
    rd = tgt - ro
    rd = (rd / np.linalg.norm(rd, axis=1, keepdims=True)).astype(np.float32)
    pg, bg = g.trace(ro, rd, False)
    po, bo, _ = o.trace(ro, rd, False)
    ntri = len(cfg4_small.model.indices)
    assert (po >= ntri).mean() > 0.3
    assert np.array_equal(pg, po)
    assert np.array_equal(bits(bg), bits(bo))
    # shadow query: octree any hit, then the shapes with the fixed tmax
    t = np.where(po >= 0, bo[:, 3], 400.0)
    tmax = (t * rng.choice([0.5, 0.999, 1.0, 1.001, 2.0], size=n)).astype(np.float32)
    og = g.occluded(ro, rd, tmax)
    assert np.array_equal(og, o.occluded(ro, rd, tmax))
    assert 0.2 < og.mean() < 0.9


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def test_shape_cull_grazing_rays_bitexact(oracle_lib):
    """The kernels skip an analytic shape's exact test when the ray segment passes outside its padded render-space
    bounding sphere (rt_device.h shape_culled, rt_host.cpp shape_bound).  Exact only if the bound holds for every
    transform: shapes under rotation and non-uniform scale (a sphere, a ring disk, a TriangleSimple), rays grazing
    their silhouettes at offsets from 1e-6 to 1e-2 of the size, rays from 1e5 away, and shadow queries ending just
    before / at / after the hit — closest hits and occlusion must be the oracle's bit for bit, with both outcomes
    present among the grazing rays."""
    cfg = scene.cfg4_mixed(res=(48, 27), spp=(2, 2), frequency=16)
    m = cfg.model
    mat = m.shapes[0].material
    S = np.diag([1.7, 0.6, 1.2, 1.0])
    sph = scene.translate((260.0, 300.0, 260.0)) @ scene.rotate(30.0, (1, 0, 0)) @ scene.rotate(45.0, (0, 1, 0)) @ S
    dsk = scene.translate((380.0, 250.0, 380.0)) @ scene.rotate(60.0, (0, 0, 1)) @ np.diag([1.3, 0.8, 1.0, 1.0])
    tri = scene.translate((120.0, 330.0, 200.0)) @ scene.rotate(20.0, (0, 1, 0))
    extra = [scene.Sphere(sph, mat, radius=40.0),
             scene.Disk(dsk, mat, height=5.0, inner_radius=12.0, outer_radius=50.0),
             scene.TriangleSimple(tri, mat, p=((0.0, 0.0, 0.0), (90.0, 10.0, 0.0), (20.0, 70.0, 30.0)))]
    m.shapes = list(m.shapes) + extra
    rng = np.random.default_rng(11)
    eps = np.array([-1e-2, -1e-4, -1e-6, 0.0, 1e-6, 1e-4, 1e-2])
    ro_all, rd_all = [], []
    for sh in extra:
        o2r = np.asarray(sh.rigid, float) @ scene.PERM_YZ
        n = 3000
        if isinstance(sh, scene.Sphere):
            u = _unit(rng.normal(size=(n, 3)))
            p = sh.radius * u * (1.0 + rng.choice(eps, n))[:, None]
            t = _unit(np.cross(u, rng.normal(size=(n, 3))))
        elif isinstance(sh, scene.Disk):
            a = rng.uniform(0, 2 * np.pi, n)
            rad = np.where(rng.random(n) < 0.5, sh.outer_radius, sh.inner_radius) * (1.0 + rng.choice(eps, n))
            p = np.stack([rad * np.cos(a), rad * np.sin(a), np.full(n, sh.height)], 1)
            t = _unit(np.stack([-np.sin(a), np.cos(a), rng.normal(scale=0.3, size=n)], 1))
        else:
            P = np.array(sh.p, float)
            i = rng.integers(0, 3, n)
            w = rng.random(n)[:, None]
            p = P[i] * (1 - w) + P[(i + 1) % 3] * w                       # on an edge
            p += _unit(rng.normal(size=(n, 3))) * rng.choice(eps, n)[:, None] * 90.0
            t = _unit(rng.normal(size=(n, 3)))
        po = p - 200.0 * t                                                 # start 200 back along the tangent
        ow = (o2r @ np.c_[po, np.ones(n)].T).T[:, :3]
        dw = _unit((o2r[:3, :3] @ t.T).T)
        far = rng.random(n) < 0.2                                           # 20 %: from 1e5 away, the same line
        ow[far] = ow[far] - 1e5 * dw[far]
        ro_all.append(ow)
        rd_all.append(dw)
    ro = np.concatenate(ro_all).astype(np.float32)
    rd = np.concatenate(rd_all).astype(np.float32)
    g, o = Renderer(cfg), oracle_lib.OracleScene(cfg)
    pg, bg = g.trace(ro, rd, False)
    po_, bo, _ = o.trace(ro, rd, False)
    ntri = len(m.indices)
    assert np.array_equal(pg, po_)
    assert np.array_equal(bits(bg), bits(bo))
    first = ntri + 4                                                       # the transformed shapes' prim ids
    hit_extra = (po_ >= first).mean()
    assert 0.15 < hit_extra < 0.85, hit_extra
    t = np.where(po_ >= 0, bo[:, 3], 1e3).astype(np.float32)
    tmax = (t * rng.choice([0.999, 1.0, 1.001, 2.0], size=len(t))).astype(np.float32)
    og = g.occluded(ro, rd, tmax)
    assert np.array_equal(og, o.occluded(ro, rd, tmax))
    assert 0.1 < og.mean() < 0.9


@pytest.mark.parametrize("kind,depth", [("path", 5), ("mis", 5), ("mis", 1), ("path", 2)])
def test_cfg4_mixed_film_bitexact(cfg4_small, oracle_lib, kind, depth):
    """Mixed scene: diffuse / mirror / BK7 glass spheres, quad + disk + point + distant lights; NEE (and MIS).
    Short depths check that the last bounce is still traced (emitters after specular bounces / with MIS)."""
    from computational_ray_tracer_amd import capi
    cfg = cfg4_small
    cfg.integrator = scene.Integrator(capi.RT_INTEGRATOR_PATH if kind == "path" else capi.RT_INTEGRATOR_PATH_MIS,
                                      max_depth=depth)
    fg = Renderer(cfg).render_pass(0, 4)
    fo = oracle_lib.OracleScene(cfg).render(0, 4)
    bad = np.any(bits(fg) != bits(fo), axis=1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ; max |diff| {np.abs(fg - fo).max()}"


@pytest.mark.parametrize("kind,depth", [("mis", 5), ("path", 2), ("mis", 1)])
def test_emitter_filter_on_off_bitexact(monkeypatch, kind, depth):
    """The last-depth emitter filter of mixed scenes (k_emitter_filter, RTMI_EMIT_FILTER, on by default) drops the
    rays that can hit no emissive surface before the last trace; its correctness rests on the closest-hit test of an
    emitter being monotone in tMax.  The film with the filter must equal the film that traces every last-depth ray,
    bit for bit (several batches on both lanes)."""
    from computational_ray_tracer_amd import capi
    cfg = scene.cfg4_mixed(res=(96, 54), spp=(2, 2), frequency=16)
    cfg.integrator = scene.Integrator(capi.RT_INTEGRATOR_PATH if kind == "path" else capi.RT_INTEGRATOR_PATH_MIS,
                                      max_depth=depth)
    monkeypatch.setenv("RTMI_BATCH_SAMPLES", str(96 * 54 * 2))
    films = {}
    for on in ("1", "0"):
        monkeypatch.setenv("RTMI_EMIT_FILTER", on)
        films[on] = Renderer(cfg).render_pass(0, 4)
    bad = np.any(bits(films["1"]) != bits(films["0"]), axis=1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ with / without the emitter filter"


def test_many_emissive_triangles_film_bitexact(oracle_lib):
    """More than kMaxEmitTris (64) emissive triangles: the emitter filter is disabled (DevScene n_emit_tris = -1) and
    the last depth traces every ray; the film still matches the oracle bit for bit.  The CFG4 mesh is made emissive
    (a Lambert material with emission, no light record: its hits count as BSDF-sampled emitter hits)."""
    from computational_ray_tracer_amd import capi
    cfg = scene.cfg4_mixed(res=(96, 54), spp=(2, 2), frequency=16)
    m = cfg.model
    mats = list(m.materials)
    glow = len(mats)
    mats.append((scene.CORNELL_WHITE, 3.0))
    m.materials = mats
    tm = np.array(m.tri_material, np.int32)
    mesh = np.arange(len(tm)) >= 12  # the box's 12 wall triangles first, then the mesh
    assert set(tm[:12].tolist()) == {0, 1, 2, 3} and set(tm[12:].tolist()) == {0} and mesh.sum() > 64
    tm[mesh] = glow
    m.tri_material = tm
    for kind in (capi.RT_INTEGRATOR_PATH_MIS, capi.RT_INTEGRATOR_PATH):
        cfg.integrator = scene.Integrator(kind, max_depth=3)
        fg = Renderer(cfg).render_pass(0, 4)
        fo = oracle_lib.OracleScene(cfg).render(0, 4)
        bad = np.any(bits(fg) != bits(fo), axis=1)
        assert bad.sum() == 0, f"{bad.sum()} pixels differ; max |diff| {np.abs(fg - fo).max()}"


@pytest.mark.parametrize("cam,filt", [("ortho", "box"), ("pinhole", "gaussian"), ("thinlens", "lanczos"),
                                      ("perspective", "gaussian"), ("perspective", "triangle")])
def test_cameras_and_filters_bitexact(oracle_lib, cam, filt):
    """Orthographic / pinhole / thin-lens cameras (Cameras.h:213-409) and the tabulated Gaussian / Lanczos
    filters (filters.h:96-264) on the CFG0 mesh, reference integrator."""
    from computational_ray_tracer_amd import capi
    base = scene.cfg0_reference(res=(48, 48), frequency=16, n_index=4)
    cams = {"ortho": scene.OrthographicCamera(near=1.0, far=2000.0, sensor=(500.0, 500.0), res=(48, 48)),
            "pinhole": scene.PinholeCamera(radius=1.0, box=(36.0, 36.0, 50.0), res=(48, 48)),
            "thinlens": scene.ThinlensCamera(curvature_radius=100.0, lens_diameter=20.0, aperture=4.0,
                                             sensor_depth=60.0, sensor=(36.0, 36.0), res=(48, 48)),
            "perspective": base.camera}
    kinds = {"box": capi.RT_FILTER_BOX, "triangle": capi.RT_FILTER_TRIANGLE, "gaussian": capi.RT_FILTER_GAUSSIAN,
             "lanczos": capi.RT_FILTER_LANCZOS}
    cfg = scene.Config("cams", base.model, cams[cam], base.sampler,
                       scene.Film(res=(48, 48), filter=kinds[filt], filter_radius=(1.0, 1.0)), base.integrator, 0, 4)
    fg = Renderer(cfg).render_pass(0, 4)
    fo = oracle_lib.OracleScene(cfg).render(0, 4)
    assert (fo[:, 0] > 0).mean() > 0.05
    assert np.array_equal(bits(fg), bits(fo))


@pytest.mark.parametrize("randomize", [0, 1, 2, 3])
def test_sobol_sampler_bitexact(oracle_lib, randomize):
    """SobolSampler (samplers.h:229-327) with the build's matrices: Cornell path mode (None / PermuteDigits /
    FastOwen / Owen), including the interval-to-index pixel mapping and the dimension wrap at 32."""
    cfg = scene.cfg_cornell(res=(48, 40), spp_side=4, max_depth=8)
    cfg.sampler = scene.SobolSampler(samples_per_pixel=16, randomize=randomize, seed=3)
    fg = Renderer(cfg).render_pass(0, 6)
    fo = oracle_lib.OracleScene(cfg).render(0, 6)
    assert np.array_equal(bits(fg), bits(fo))


def _cornell_surface_rays(model, rng, per_tri=64):
    """Waves of 64 rays leaving one triangle of the Cornell box: origins on the surface offset along the normal by
    0, the path integrator's 1e-4 (1 + max|p|), and values either side of the cluster-box pad; directions in the
    hemisphere (so the waves are direction-coherent and exercise the cluster skipping of both traversals)."""
    P = model.positions.astype(np.float64)[model.indices.astype(np.int64)][..., [0, 2, 1]]  # object -> world (perm_yz)
    ro, rd = [], []
    for t in range(len(P)):
        a, b, c = P[t]
        n = np.cross(b - a, c - a)
        n /= np.linalg.norm(n)
        u, v = rng.random(per_tri), rng.random(per_tri)
        flip = u + v > 1
        u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
        p = a + u[:, None] * (b - a) + v[:, None] * (c - a)
        off = rng.choice([0.0, 1e-6, -1e-4, 1e-3, 0.006, 0.0066, 0.0072, 0.05], size=per_tri)
        nee = 1e-4 * (1 + np.abs(p).max(axis=1))
        off = np.where(rng.random(per_tri) < 0.5, nee, off)
        for s in (1.0, -1.0):  # both sides of the surface
            d = rng.normal(size=(per_tri, 3))
            d *= np.sign(d @ (s * n))[:, None]
            d /= np.linalg.norm(d, axis=1, keepdims=True)
            ro.append(p + (s * off)[:, None] * n)
            rd.append(d)
    return np.concatenate(ro).astype(np.float32), np.concatenate(rd).astype(np.float32)


def test_cornell_surface_rays_closest_and_occluded_bitexact(oracle_lib):
    """Closest-hit and shadow (any-hit) queries from the box's own surfaces, in direction-coherent waves: the
    single-leaf two-pass test, fan-pair vertex sharing and conservative cluster skipping must not change a bit."""
    cfg = scene.cfg_cornell(res=(32, 32), spp_side=1)
    g, o = Renderer(cfg), oracle_lib.OracleScene(cfg)
    rng = np.random.default_rng(11)
    ro, rd = _cornell_surface_rays(cfg.model, rng)
    pg, bg = g.trace(ro, rd, False)
    po, bo, _ = o.trace(ro, rd, False)
    assert np.array_equal(pg, po)
    assert np.array_equal(bits(bg), bits(bo))
    assert (pg >= 0).mean() > 0.4
    # shadow queries: towards points on the light quad (tmax = 0.999 dist, as the integrator) and random tmax
    L = cfg.model.lights[0]
    u, v = rng.random(len(ro)), rng.random(len(ro))
    tgt = np.asarray(L["p"]) + u[:, None] * np.asarray(L["e1"]) + v[:, None] * np.asarray(L["e2"])
    w = tgt - ro.astype(np.float64)
    dist = np.linalg.norm(w, axis=1)
    sd = (w / dist[:, None]).astype(np.float32)
    tmax = np.where(rng.random(len(ro)) < 0.7, 0.999 * dist, rng.random(len(ro)) * 800).astype(np.float32)
    og = g.occluded(ro, sd, tmax)
    oo = o.occluded(ro, sd, tmax)
    assert np.array_equal(og, oo)
    assert 0.05 < og.mean() < 0.95
    og2 = g.occluded(ro, rd, tmax)
    assert np.array_equal(og2, o.occluded(ro, rd, tmax))


@pytest.mark.parametrize("sensor,illum", [(0, 1), (1, 1), (9, 0), (17, 2)])
def test_pixel_sensor_film_and_resolve_bitexact(oracle_lib, sensor, illum):
    """XYZ sensor under another illuminant and camera-curve sensors (pixelsensor.h:37-87): the film kernel's
    sensor curves, the host's XYZFromSensorRGB and the resolve bytes all equal the oracle's."""
    cfg = scene.cfg_cornell(res=(48, 32), spp_side=2)
    cfg.film.sensor, cfg.film.sensor_illum = sensor, illum
    g, o = Renderer(cfg), oracle_lib.OracleScene(cfg)
    ga, gb = g.film_matrices()
    oa, ob = o.resolve_matrices()
    assert np.array_equal(bits(ga), bits(oa)) and np.array_equal(bits(gb), bits(ob))
    fg = g.render_pass(0, 4)
    fo = o.render(0, 4)
    assert np.array_equal(bits(fg), bits(fo))
    assert np.array_equal(g.resolve(fg), o.resolve(fo))
    assert np.array_equal(g.resolve(fg, srgb=True), o.resolve(fo, srgb=True))


def test_pixel_sensor_reference_integrator_bitexact(oracle_lib):
    cfg = scene.cfg0_reference(res=(64, 64), frequency=16, n_index=3)
    cfg.film.sensor, cfg.film.sensor_illum = capi.RT_SENSOR_CANON_EOS_100D, capi.RT_ILLUM_A
    g, o = Renderer(cfg), oracle_lib.OracleScene(cfg)
    fg = g.render_pass(0, 3)
    fo = o.render(0, 3)
    assert np.array_equal(bits(fg), bits(fo))


def _soup_config(pos, capacity):
    n = len(pos) // 3
    m = scene.TriModel(pos.astype(np.float32), np.tile([0, 0, 1], (len(pos), 1)).astype(np.float32),
                       np.arange(len(pos), dtype=np.uint32).reshape(n, 3), rigid=np.eye(4) @ scene.PERM_YZ,
                       octree_capacity=capacity, tri_material=np.zeros(n, np.int32))
    m.materials = [(scene.grey_sigmoid(0.5), 0.0)]
    return scene.Config("soup", m, scene.cornell_camera((8, 8)), scene.StratifiedSampler(1, 1, True, 0),
                        scene.Film(res=(8, 8)), scene.Integrator(capi.RT_INTEGRATOR_PATH, max_depth=2), 0, 1)


def _soups():
    rng = np.random.default_rng(21)
    out = []
    # random triangle soup (small and large triangles) at several capacities
    c = rng.uniform(0, 100, (3000, 1, 3))
    soup = c + rng.normal(size=(3000, 3, 3)) * rng.choice([0.5, 5.0, 30.0], (3000, 1, 1))
    out += [(soup[rng.random(3000) < 0.3][:600] / 3, 4), (soup, 40)]
    # clustered: 300 copies of one tiny triangle among a few hundred others -> repeated aborted splits
    tiny = np.array([[[10, 10, 10], [10.01, 10, 10], [10, 10.01, 10]]]).repeat(300, 0)
    other = rng.uniform(0, 50, (400, 1, 3)) + rng.normal(size=(400, 3, 3))
    mix = np.concatenate([other[:200], tiny, other[200:]])
    out.append((mix, 40))
    # axis-aligned grid of quads (ties on child-box boundaries)
    g = []
    for i in range(30):
        for j in range(30):
            a, b, cc, d = [i, j, 0], [i + 1, j, 0], [i + 1, j + 1, 0], [i, j + 1, 0]
            g += [[a, b, cc], [a, cc, d]]
    out.append((np.array(g, float) * 3.0, 8))
    return out


@pytest.mark.parametrize("case", range(4))
def test_device_octree_build_equals_sequential(oracle_lib, case):
    """rt_options.octree_build: the level-synchronous device build (rt_octree.hip) reproduces the reference's
    insertion-order tree — same nodes, same numbering, same leaf lists — as the host's sequential build and the
    oracle, including aborted splits, tiny capacities and triangles on child-box boundaries."""
    tris, cap = _soups()[case]
    cfg = _soup_config(tris.reshape(-1, 3)[:, [0, 2, 1]], cap)   # object space = world with y/z swapped
    gd = Renderer(cfg, octree_build=capi.RT_OCTREE_BUILD_DEVICE).octree()
    gh = Renderer(cfg, octree_build=capi.RT_OCTREE_BUILD_HOST).octree()
    go = oracle_lib.OracleScene(cfg).octree()
    for a in (gh, go):
        assert np.array_equal(bits(gd["bounds"]), bits(a["bounds"]))
        assert np.array_equal(gd["child"], a["child"])
        assert np.array_equal(gd["leaf_count"], a["leaf_count"])
        assert np.array_equal(gd["refs"], a["refs"])
    assert len(gd["child"]) > 9


def test_device_octree_build_cfg3_matches_host(cfg3_pair):
    import time
    cfg, gdev, _ = cfg3_pair
    t0 = time.perf_counter()
    gh = Renderer(cfg, octree_build=capi.RT_OCTREE_BUILD_HOST)
    t_host = time.perf_counter() - t0
    t0 = time.perf_counter()
    gd = Renderer(cfg, octree_build=capi.RT_OCTREE_BUILD_DEVICE)
    t_dev = time.perf_counter() - t0
    a, b = gd.octree(), gh.octree()
    for k in ("bounds", "child", "leaf_count", "refs"):
        assert np.array_equal(bits(a[k]) if k == "bounds" else a[k], bits(b[k]) if k == "bounds" else b[k])
    print(f"\nCFG3 scene upload: host build {t_host * 1e3:.0f} ms, device build {t_dev * 1e3:.0f} ms")


@pytest.mark.parametrize("kind,ndev", [("cornell", 2), ("cornell", 3), ("mesh", 2), ("reference", 3)])
def test_multi_device_context_film_bitexact(oracle_lib, kind, ndev):
    """rt_options.devices (SURVEY §8b device list): one context rendering on several devices, pixel tiles
    interleaved, owned pixels exchanged by peer copies.  On the 1-GPU test box device 0 is listed `ndev` times
    (separate contexts, streams and buffers on one GPU): the same code path as distinct GPUs.  The film —
    accumulated over two passes, so the exchange must carry the caller's earlier values — is bit-identical to
    the oracle (tolerance 0)."""
    if kind == "cornell":
        cfg = scene.cfg_cornell(res=(72, 40), spp_side=2)
    elif kind == "mesh":
        cfg = scene.cfg3_blob(res=(64, 40), spp_side=2, max_depth=3, frequency=20)
    else:
        cfg = scene.cfg0_reference(res=(64, 64), frequency=8, n_index=4)
    g = Renderer(cfg, device=[0] * ndev)
    f = g.new_film()
    g.render_pass(0, 1, f)
    g.render_pass(1, 4, f)
    fo = oracle_lib.OracleScene(cfg).render(0, 4)
    bad = np.any(bits(f) != bits(fo), axis=1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ"
    st = g.stats()
    assert st["samples"] == 4 * cfg.film.res[0] * cfg.film.res[1]   # summed over the devices


def test_multi_device_device_film_and_shard(oracle_lib):
    """Device-resident film (rt_render_pass_device) on a 2-device context, and a process-level shard split
    over the context's devices: equals the single-device render of the same shard."""
    import torch
    cfg = scene.cfg_cornell(res=(80, 48), spp_side=2)
    one = Renderer(cfg)
    one.set_shard(16, 2, 1)
    ref = one.render_pass(0, 4)
    g = Renderer(cfg, device=[0, 0])
    g.set_shard(16, 2, 1)
    film = torch.zeros((80 * 48, 4), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    g.render_pass_device(0, 2, film.data_ptr(), s.cuda_stream)
    g.render_pass_device(2, 4, film.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(bits(film.cpu().numpy()), bits(ref))


@pytest.mark.parametrize("kind,i0,i1", [("cornell", 0, 2), ("cornell", 254, 256), ("cfg3", 510, 512),
                                         ("cfg4", 1022, 1024), ("cfg4", 300, 303), ("cfg5", 2046, 2048)])
def test_full_size_workload_sampled_pixels_bitexact(oracle_lib, kind, i0, i1):
    """BASELINE configs[1]-[4] at their full size (1080p / 4K, 256-2048 spp strata) over the first or last
    sample indices of the frame: the GPU renders every pixel, the oracle a seeded sample of 4096 of them (16384 on
    the mixed scenes)
    (bit-exact there), and the rest is checked through size-independent properties: a pass split into two
    accumulates to the same bits, every film value is finite and non-negative, every rendered pixel carries
    the same filter weight."""
    cfg = {"cornell": lambda: scene.cfg_cornell(res=(1920, 1080), spp_side=16), "cfg3": scene.cfg3_blob,
           "cfg4": scene.cfg4_mixed, "cfg5": scene.cfg5_spectral}[kind]()
    g = Renderer(cfg)
    fg = g.render_pass(i0, i1)
    npx = cfg.film.res[0] * cfg.film.res[1]
    n_check = 16384 if kind in ("cfg4", "cfg5") else 4096  # the branchy mixed scenes get a larger sample
    pix = np.sort(np.random.default_rng(7).choice(npx, n_check, replace=False)).astype(np.int32)
    fo = oracle_lib.OracleScene(cfg).render(i0, i1, pixel_ids=pix)
    assert np.array_equal(bits(fg[pix]), bits(fo[pix]))
    f2 = g.new_film()
    g.render_pass(i0, i0 + 1, f2)
    g.render_pass(i0 + 1, i1, f2)
    assert np.array_equal(bits(f2), bits(fg))
    assert np.all(np.isfinite(fg)) and np.all(fg >= 0)
    assert np.all(fg[:, 3] == fg[0, 3]) and fg[0, 3] > 0
    assert g.stats()["samples"] >= npx * (i1 - i0)


@pytest.mark.parametrize("kind", ["path", "reference"])
def test_independent_sampler_bitexact(oracle_lib, kind):
    """IndependentSampler (samplers.h:38-62: PCG32 per pixel, Advance(index·65536 + dim), every Get1D/Get2D a
    fresh draw) on the Cornell path integrator and on the CFG0 reference integrator: films and, in reference mode,
    the per-sample records (λ, pdf, ray, hit, L, rgb) bit-exact (tolerance 0)."""
    if kind == "path":
        cfg = scene.cfg_cornell(res=(48, 40), spp_side=2)
    else:
        cfg = scene.cfg0_reference(res=(64, 64), frequency=16, n_index=5)
    cfg.sampler = scene.IndependentSampler(samples_per_pixel=7, seed=3)
    g, o = Renderer(cfg), oracle_lib.OracleScene(cfg)
    fg = g.render_pass(0, 5)
    fo = o.render(0, 5)
    assert np.array_equal(bits(fg), bits(fo))
    if kind == "reference":
        rng = np.random.default_rng(2)
        pix = rng.integers(0, 64 * 64, 4000)
        idx = rng.integers(0, 50, 4000)          # indices beyond spp are fine for the independent sampler
        a = records_to_arrays(g.samples(pix, idx))
        b = records_to_arrays(o.samples(pix, idx))
        for k in a:
            assert np.array_equal(bits(a[k]), bits(b[k])), k


def _triangle_simple_scene():
    """Cornell box + two TriangleSimple shapes (Shapes.h:760-907): one floating in the box, one in the back wall's
    plane (world z = 559.2: object y, Shapes.h:178), so rays to the back wall hit both at (nearly) the same t and
    the shape's `t >= tMax` rejection (Shapes.h:866) decides against it on ties."""
    cfg = scene.cfg_cornell(res=(48, 40), spp_side=2)
    m = cfg.model
    mats = list(m.materials)
    mid = len(mats)
    mats.append((scene.CORNELL_RED, 0.0, capi.RT_MAT_DIFFUSE, 0.0))
    m.materials = mats
    m.shapes = [scene.TriangleSimple(scene.translate((0.0, 0.0, 0.0)), mid,
                                     p=((150.0, 250.0, 200.0), (420.0, 300.0, 260.0), (260.0, 200.0, 470.0))),
                scene.TriangleSimple(np.eye(4), mid, p=((100.0, 559.2, 100.0), (400.0, 559.2, 100.0),
                                                         (250.0, 559.2, 450.0)))]
    cfg.integrator = scene.Integrator(capi.RT_INTEGRATOR_PATH_MIS, max_depth=4)
    return cfg


def test_triangle_simple_trace_and_film_bitexact(oracle_lib):
    cfg = _triangle_simple_scene()
    g, o = Renderer(cfg), oracle_lib.OracleScene(cfg)
    ntri = len(cfg.model.indices)
    rng = np.random.default_rng(9)
    n = 30000
    ro = np.stack([rng.uniform(5, 550, n), rng.uniform(5, 543, n), rng.uniform(5, 300, n)], 1).astype(np.float32)
    tgt = np.where(rng.random((n, 1)) < 0.5,
                   np.c_[rng.uniform(100, 400, n), rng.uniform(100, 450, n), np.full(n, 559.2)],   # back wall
                   np.c_[rng.uniform(150, 420, n), rng.uniform(200, 300, n), rng.uniform(200, 470, n)])
    rd = tgt - ro
    rd = (rd / np.linalg.norm(rd, axis=1, keepdims=True)).astype(np.float32)
    pg, bg = g.trace(ro, rd, False)
    po, bo, _ = o.trace(ro, rd, False)
    assert (po == ntri).mean() > 0.1           # the floating TriangleSimple
    assert np.array_equal(pg, po)
    assert np.array_equal(bits(bg), bits(bo))
    t = np.where(po >= 0, bo[:, 3], 400.0)
    tmax = (t * rng.choice([0.5, 0.999, 1.0, 1.001, 2.0], size=n)).astype(np.float32)
    assert np.array_equal(g.occluded(ro, rd, tmax), o.occluded(ro, rd, tmax))
    fg = g.render_pass(0, 4)
    fo = o.render(0, 4)
    assert np.array_equal(bits(fg), bits(fo))


def test_bvh_fast_path_counters(cfg3_pair):
    """Multi-level scenes trace through the BVH: executed box / triangle tests per ray far below
    the reference BFS's, and the BFS fallback reserved to the rare ambiguous rays."""
    cfg, g, _ = cfg3_pair
    g.reset_stats()
    g.render_pass(0, 2)
    st = g.stats()
    assert st["rays"] > 0 and st["shadow_rays"] > 0
    assert st["tris_tested"] / st["rays"] < 12, st
    assert st["fallback_rays"] <= 1e-3 * st["rays"], st
    assert st["shadow_fallback_rays"] <= 1e-2 * st["shadow_rays"], st
    assert st["coop_overflows"] == 0, st


@pytest.mark.parametrize("nl,single_leaf", [(1, False), (2, True), (6, False), (6, True)])
def test_deferred_nee_light_counts_bitexact(oracle_lib, nl, single_leaf):
    """Deferred NEE (k_path_shade_full -> k_path_nee) with 1, 2 and 6 lights: NEE records of nee_stride(n) float4
    (the light weights spill into a second float4 at 6 lights), light order kept per vertex; MIS on; a 3 x 3
    stratified sampler (the non-power-of-two sampler path) on an odd film; single-leaf (Cornell box + spheres,
    one shard, static chunks) and multi-level (the CFG4 mesh, 8 shards, tickets) scenes."""
    import copy
    from computational_ray_tracer_amd import capi
    res = (37, 23)
    base = scene.cfg4_mixed(res=res, spp=(3, 3), frequency=16)
    m = copy.deepcopy(base.model)
    if single_leaf:  # the box without the mesh: 12 triangles, one leaf; the shapes make it a mixed scene
        cb = scene.cornell_box(blocks=False)
        m.positions, m.normals, m.indices = cb.positions, cb.normals, cb.indices
        m.tri_material = cb.tri_material
    extra = [dict(type=capi.RT_LIGHT_POINT, p=(100.0 + 60 * k, 380.0, 200.0 + 40 * k), scale=1.0e4 * (k + 1))
             for k in range(4)]
    lights = list(m.lights) + extra
    m.lights = lights[:nl]
    cfg = scene.Config(f"nee{nl}", m, base.camera, scene.StratifiedSampler(3, 3, True, 0), base.film,
                       scene.Integrator(capi.RT_INTEGRATOR_PATH_MIS, max_depth=4), 0, 9)
    r = Renderer(cfg)
    assert (r.octree()["depth"] == 0) == single_leaf
    fg = r.render_pass(0, 3)
    fo = oracle_lib.OracleScene(cfg).render(0, 3)
    bad = np.any(bits(fg) != bits(fo), axis=1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ; max |diff| {np.abs(fg - fo).max()}"
    assert r.stats()["shadow_rays"] > 0


@pytest.mark.parametrize("spec", ["0", "1", "1/3"])
def test_nee_morton_sort_bitexact(oracle_lib, monkeypatch, spec):
    """RTMI_SORT_NEE: the NEE queue of a multi-level mixed scene reordered by the Morton code of the shading points
    (rt_sort.hip k_nee_keys / k_nee_scatter) before k_path_nee; vertices are independent and each keeps its light
    order, so the film stays bit-exact (6 lights, several batches on both lanes)."""
    import copy
    from computational_ray_tracer_amd import capi
    monkeypatch.setenv("RTMI_SORT_NEE", spec)
    monkeypatch.setenv("RTMI_BATCH_SAMPLES", str(37 * 23 * 2))
    monkeypatch.setenv("RTMI_LANES", "2")
    res = (37, 23)
    base = scene.cfg4_mixed(res=res, spp=(3, 3), frequency=16)
    m = copy.deepcopy(base.model)
    extra = [dict(type=capi.RT_LIGHT_POINT, p=(100.0 + 60 * k, 380.0, 200.0 + 40 * k), scale=1.0e4 * (k + 1))
             for k in range(4)]
    m.lights = (list(m.lights) + extra)[:6]
    cfg = scene.Config("nee_sort", m, base.camera, scene.StratifiedSampler(3, 3, True, 0), base.film,
                       scene.Integrator(capi.RT_INTEGRATOR_PATH_MIS, max_depth=4), 0, 9)
    r = Renderer(cfg)
    assert r.octree()["depth"] > 0
    fg = r.render_pass(0, 7)
    fo = oracle_lib.OracleScene(cfg).render(0, 7)
    bad = np.any(bits(fg) != bits(fo), axis=1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ; max |diff| {np.abs(fg - fo).max()}"
    st = r.stats()
    assert st["shadow_rays"] > 0 and st["ms_sort"] > 0


def _cornell_edge_rays(cfg, rng):
    """Rays that put an edge function of the single-leaf test exactly at 0: axis-parallel rays through every vertex
    of the Cornell box (after the watertight test's translation the vertex sits at the origin of the sheared frame),
    and through points of its axis-aligned edges, interleaved with random rays so that waves mix dominant axes (the
    compacted pass 1) as well as share one (the ballot path)."""
    from test_canonical_traversal import _world_tris
    tris = _world_tris(cfg.model).astype(np.float32)
    verts = np.unique(tris.reshape(-1, 3), axis=0)
    lo, hi = verts.min(0), verts.max(0)
    c = (lo + hi) / 2
    ro, rd = [], []
    for v in verts:
        for ax in range(3):
            for sgn in (1.0, -1.0):
                d = np.zeros(3, np.float32)
                d[ax] = sgn
                o = v.copy()
                o[ax] = c[ax] - sgn * 0.25 * (hi[ax] - lo[ax])   # inside the box, the ray passes through v
                ro.append(o); rd.append(d)
    for t in tris:                                           # points on the edges (midpoints, quarter points)
        for a, b in ((0, 1), (1, 2), (2, 0)):
            for f in (0.25, 0.5):
                p = (t[a] + np.float32(f) * (t[b] - t[a])).astype(np.float32)
                ax = int(np.argmax(np.abs(p - c)))
                d = np.zeros(3, np.float32)
                d[ax] = 1.0 if p[ax] > c[ax] else -1.0
                o = p.copy()
                o[ax] = c[ax]
                ro.append(o); rd.append(d)
    ro, rd = np.array(ro, np.float32), np.array(rd, np.float32)
    by_axis = np.argsort(np.argmax(np.abs(rd), 1), kind="stable")   # waves sharing a dominant axis: the ballot path
    ro, rd = ro[by_axis], rd[by_axis]
    n = len(ro)
    rr = (c + (rng.random((n, 3)) - 0.5) * (hi - lo) * 0.9).astype(np.float32)
    dd = rng.normal(size=(n, 3)).astype(np.float32)
    dd /= np.linalg.norm(dd, axis=1, keepdims=True)
    mix_o, mix_d = np.empty((2 * n, 3), np.float32), np.empty((2 * n, 3), np.float32)
    mix_o[0::2], mix_d[0::2], mix_o[1::2], mix_d[1::2] = ro, rd, rr, dd
    return np.concatenate([ro, mix_o]), np.concatenate([rd, mix_d])


def test_single_leaf_vertex_and_edge_rays_bitexact(oracle_lib):
    """Round 6 changed the single-leaf tests: the candidate filter keeps a triangle with an exactly-zero edge for the
    exact pass 2 (no double recompute), and shadow rays walk their own hit clusters per lane.  Rays through vertices
    and along edges of the Cornell box (zero edges by construction) must still match the oracle bit for bit, for
    closest hit and for the any-hit query at the hit distance x {0.5, 0.999, 1, 1.001, 2} (tolerance 0)."""
    cfg = scene.cfg_cornell(res=(32, 32), spp_side=1)
    g, o = Renderer(cfg), oracle_lib.OracleScene(cfg)
    ro, rd = _cornell_edge_rays(cfg, np.random.default_rng(11))
    pg, bg = g.trace(ro, rd, True)
    po, bo, _ = o.trace(ro, rd, True)
    assert (po >= 0).mean() > 0.5
    assert np.array_equal(pg, po)
    assert np.array_equal(bits(bg), bits(bo))
    hit = po >= 0
    for f in (0.5, 0.999, 1.0, 1.001, 2.0):
        tm = (bo[hit, 3] * np.float32(f)).astype(np.float32)
        og = g.occluded(ro[hit], rd[hit], tm)
        oo = o.occluded(ro[hit], rd[hit], tm)
        assert np.array_equal(np.asarray(og, bool), np.asarray(oo, bool)), f
