"""CPU: pin the oracle (the C++ restatement of the reference path) against known answers.

The reference ships no tests, fixtures or golden files and cannot be compiled here
(SURVEY.md §8c), so the oracle is pinned by (i) published external vectors (PCG32 demo output),
(ii) independent pure-Python restatements of the published integer algorithms, and (iii) the analytic
known answers listed in SURVEY.md §8c (numbered as there).
"""
import ctypes as C
import math

import numpy as np
import pytest

from computational_ray_tracer_amd import capi, scene

M64 = (1 << 64) - 1


def fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


# ------------------------------------------------------------------------ independent Python restatements
def py_pcg_step(state, inc):
    old = state
    state = (old * 0x5851F42D4C957F2D + inc) & M64
    xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
    rot = old >> 59
    return state, ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF


def py_murmur64a(key: bytes, seed=0):
    m, r = 0xC6A4A7935BD1E995, 47
    h = (seed ^ (len(key) * m)) & M64
    nblocks = len(key) // 8
    for i in range(nblocks):
        k = int.from_bytes(key[8 * i: 8 * i + 8], "little")
        k = (k * m) & M64
        k ^= k >> r
        k = (k * m) & M64
        h ^= k
        h = (h * m) & M64
    tail = key[8 * nblocks:]
    if tail:
        for i in reversed(range(len(tail))):
            h ^= tail[i] << (8 * i)
        h = (h * m) & M64
    h ^= h >> r
    h = (h * m) & M64
    h ^= h >> r
    return h


def py_mixbits(v):
    v ^= v >> 31
    v = (v * 0x7FB5D329728EA185) & M64
    v ^= v >> 27
    v = (v * 0x81DADEF4BC2DD44D) & M64
    v ^= v >> 33
    return v


# ------------------------------------------------------------------------------------------ (1) PCG32
def test_pcg32_published_demo_vector(oracle_lib):
    """pcg32_srandom(42, 54) — the PCG reference demo output (pcg-random.org, pcg32-demo)."""
    out = np.zeros(6, np.uint32)
    oracle_lib.lib().orc_pcg_draws(2, 54, 42, 6, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    assert [hex(v) for v in out] == ["0xa15c02b7", "0x7b47f409", "0xba1d3330", "0x83d2f293", "0xbfa4784b", "0xcbed606e"]


def test_pcg32_default_state_matches_python(oracle_lib):
    out = np.zeros(64, np.uint32)
    oracle_lib.lib().orc_pcg_draws(0, 0, 0, 64, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    st, inc = 0x853C49E6748FEA9B, 0xDA3E39CB94B95BDB
    ref = []
    for _ in range(64):
        st, v = py_pcg_step(st, inc)
        ref.append(v)
    assert out.tolist() == ref


@pytest.mark.parametrize("seq", [0, 1, 12345678901234, (1 << 63) + 17])
@pytest.mark.parametrize("adv", [0, 1, 7, 65536, 3 * 65536 + 5, 255 * 65536 + 4])
def test_pcg32_advance_equals_draws(oracle_lib, seq, adv):
    """rng.h:131-144 Advance(n) lands on the same state as n sequential draws (SetSequence via MixBits)."""
    L = oracle_lib.lib()
    a = np.zeros(4, np.uint32)
    L.orc_pcg_draws(1, seq, adv, 4, a.ctypes.data_as(C.POINTER(C.c_uint32)))
    inc = ((seq << 1) | 1) & M64
    st = 0
    st, _ = py_pcg_step(st, inc)
    st = (st + py_mixbits(seq)) & M64
    st, _ = py_pcg_step(st, inc)
    # jump by repeated squaring in Python (independent of the C++ loop)
    mult, plus, am, ap, d = 0x5851F42D4C957F2D, inc, 1, 0, adv
    while d:
        if d & 1:
            am = (am * mult) & M64
            ap = (ap * mult + plus) & M64
        plus = ((mult + 1) * plus) & M64
        mult = (mult * mult) & M64
        d >>= 1
    st = (am * st + ap) & M64
    ref = []
    for _ in range(4):
        st, v = py_pcg_step(st, inc)
        ref.append(v)
    assert a.tolist() == ref
    if adv <= 70000:  # and equals literally drawing adv values
        st2 = 0
        st2, _ = py_pcg_step(st2, inc)
        st2 = (st2 + py_mixbits(seq)) & M64
        st2, _ = py_pcg_step(st2, inc)
        for _ in range(adv):
            st2, _ = py_pcg_step(st2, inc)
        _, v0 = py_pcg_step(st2, inc)
        assert v0 == ref[0]


# ------------------------------------------------------------------------------------ (2) hashing
def test_murmur64a_matches_python(oracle_lib):
    L = oracle_lib.lib()
    rng = np.random.default_rng(0)
    for n in list(range(0, 33)) + [100, 257]:
        key = rng.integers(0, 256, n, dtype=np.uint8)
        for seed in (0, 1, 0xDEADBEEF12345678):
            got = L.orc_murmur64a(key.ctypes.data_as(C.POINTER(C.c_uint8)), n, seed)
            assert got == py_murmur64a(key.tobytes(), seed)


def test_mixbits_and_pixel_hash_keys(oracle_lib):
    L = oracle_lib.lib()
    for v in (0, 1, 2 ** 63, 0x0123456789ABCDEF, M64):
        assert L.orc_mixbits(v) == py_mixbits(v)
    # hash.h:96-104: Hash(ivec2, int) hashes the 12-byte packed key; Hash(ivec2, int, int) the 16-byte one
    for x, y, d, s in ((0, 0, 0, 0), (17, 499, 3, 0), (-1, 5, 7, 42), (1919, 1080, 12, 7)):
        k12 = np.array([x, y, s], np.int32).tobytes()
        k16 = np.array([x, y, d, s], np.int32).tobytes()
        assert L.orc_hash_pixel(x, y, s) == py_murmur64a(k12)
        assert L.orc_hash_pixel_dim(x, y, d, s) == py_murmur64a(k16)


# ------------------------------------------------------------------------------ (3) PermutationElement
@pytest.mark.parametrize("l", [1, 2, 16, 100, 256, 1000])
def test_permutation_element_is_bijection(oracle_lib, l):
    L = oracle_lib.lib()
    for p in (0, 1, 0xDEADBEEF, 0x12345678):
        vals = sorted(L.orc_permutation_element(i, l, p) for i in range(l))
        assert vals == list(range(l))


# ------------------------------------------------------------------------ (4) stratified sampler grid
def test_stratified_no_jitter_covers_grid(oracle_lib):
    L = oracle_lib.lib()
    d = capi.rt_sampler_desc(capi.RT_SAMPLER_STRATIFIED, 10, 10, 0, 0)
    ops = (C.c_int * 3)(1, 2, 2)
    u1, u2 = [], []
    for idx in range(100):
        out = (C.c_float * 5)()
        assert L.orc_sampler_draws(C.byref(d), 37, 201, idx, 3, ops, out) == 5
        u1.append(out[0])
        u2.append((out[1], out[2]))
    assert sorted(u1) == [np.float32((s + 0.5) / 100) for s in range(100)]
    grid = sorted((np.float32((x + 0.5) / 10), np.float32((y + 0.5) / 10)) for x in range(10) for y in range(10))
    assert sorted(u2) == grid
    # StratifiedSampler without jitter refuses index >= spp (samplers.h:83-87)
    out = (C.c_float * 5)()
    assert L.orc_sampler_draws(C.byref(d), 0, 0, 100, 3, ops, out) == -1


def test_stratified_jitter_stays_in_strata(oracle_lib):
    L = oracle_lib.lib()
    d = capi.rt_sampler_desc(capi.RT_SAMPLER_STRATIFIED, 4, 4, 1, 0)
    ops = (C.c_int * 1)(2)
    cells = set()
    for idx in range(16):
        out = (C.c_float * 2)()
        L.orc_sampler_draws(C.byref(d), 3, 9, idx, 1, ops, out)
        cells.add((int(out[0] * 4), int(out[1] * 4)))
    assert len(cells) == 16


# --------------------------------------------------------------------------- (5) visible wavelengths
def test_visible_wavelength_pdf_and_inverse(oracle_lib):
    L = oracle_lib.lib()
    lam = np.linspace(360, 830, 47001)
    pdf = np.array([L.orc_visible_pdf(float(x)) for x in lam[::10]], np.float64)
    integral = np.trapezoid(pdf, lam[::10])
    assert abs(integral - 1.0) < 2e-3
    assert L.orc_visible_pdf(359.0) == 0 and L.orc_visible_pdf(831.0) == 0
    # inverse CDF: CDF(lambda(u)) = u with the analytic CDF of 0.0039398042 / cosh^2(0.0072 (l - 538))
    A, B = 0.0039398042, 0.0072
    cdf = lambda l: (A / B) * (math.tanh(B * (l - 538)) - math.tanh(B * (360 - 538)))
    for u in (0.01, 0.1, 0.25, 0.5, 0.75, 0.9, 0.99):
        lu = L.orc_sample_visible_wavelength(u)
        assert 360 <= lu <= 830
        assert abs(cdf(lu) - u) < 2e-3


def test_sample_visible_hero_offsets(oracle_lib):
    """spectrum.h:322-336: 8 wavelengths at up = u + i/8 (wrapped)."""
    L = oracle_lib.lib()
    lam, pdf = np.zeros(8, np.float32), np.zeros(8, np.float32)
    L.orc_sample_visible(np.float32(0.3), fp(lam), fp(pdf))
    for i in range(8):
        up = np.float32(np.float32(0.3) + np.float32(i) / np.float32(8))
        if up > 1:
            up = np.float32(up - 1)
        assert lam[i] == np.float32(L.orc_sample_visible_wavelength(float(up)))
        assert pdf[i] == np.float32(L.orc_visible_pdf(float(lam[i])))


# ---------------------------------------------------------------------------------- (6)-(8) spectra
def test_spectra_init_normalisation(oracle_lib):
    L = oracle_lib.lib()
    # spectrum.cpp:162: FromInterleaved(normalize) scales so InnerProduct(s, Y) = CIE_Y_integral
    assert abs(L.orc_inner_product_y_d65() - 106.856895) / 106.856895 < 1e-4
    X, Y, Z, D = (np.zeros(471, np.float32) for _ in range(4))
    L.orc_spectra_dense(fp(X), fp(Y), fp(Z), fp(D))
    # CIE 1931 Y peaks at 555 nm with value 1.0; dense tables are the piecewise data at integer nm
    assert int(np.argmax(Y)) + 360 == 555 and Y.max() == np.float32(1.0)
    # D65 dense == normalized piecewise D65 queried at integer nm (spectrum.h:412-419)
    q = np.zeros(471, np.float32)
    L.orc_spectra_query(0, 471, fp(np.arange(360, 831, dtype=np.float32)), fp(q))
    assert np.array_equal(q, D)


def test_grey_sigmoid_and_illuminant_branch(oracle_lib):
    """color.cpp:35-37: RGB(.5,.5,.5) -> c2 = 0 -> s(0) = 0.5 at every wavelength."""
    L = oracle_lib.lib()
    c = scene.grey_sigmoid(0.5)
    assert c == (0.0, 0.0, 0.0)
    for lam in (360.0, 500.0, 830.0):
        assert L.orc_sigmoid_eval(0.0, 0.0, 0.0, lam) == 0.5
    c = scene.grey_sigmoid(0.73)
    assert abs(L.orc_sigmoid_eval(*c, 600.0) - 0.73) < 1e-6


def test_srgb_white_maps_to_d65(oracle_lib):
    """(7) colorspace.cpp:13-28: XYZFromRGB * (1,1,1) = the D65 white; the resolve maps an all-white sensor
    film to (255, 255, 255) up to the Bradford round trip."""
    cfg = scene.cfg0_reference(res=(4, 4), frequency=2, n_index=1)
    o = oracle_lib.OracleScene(cfg)
    film = np.ones((16, 4), np.float32)
    A, B = np.zeros(9, np.float32), np.zeros(9, np.float32)
    oracle_lib.lib().orc_resolve_matrices(o.h, fp(A), fp(B))
    XYZ_from_sensor = A.reshape(3, 3).T
    RGB_from_XYZ = B.reshape(3, 3).T
    assert np.allclose(XYZ_from_sensor, np.eye(3), atol=2e-3)
    xyz_white = np.linalg.inv(RGB_from_XYZ) @ np.ones(3)
    assert abs(xyz_white[1] - 1.0) < 1e-4
    assert abs(xyz_white[0] / xyz_white.sum() - 0.3127) < 2e-3 and abs(xyz_white[1] / xyz_white.sum() - 0.3290) < 2e-3
    # the XYZ sensor film holding the D65 white resolves to sRGB white (XYZ(1,1,1) would not: E != D65)
    film[:, :3] = (np.linalg.inv(XYZ_from_sensor) @ xyz_white).astype(np.float32)
    assert (o.resolve(film) >= 253).all()


# -------------------------------------------------------------------------------- (9) watertight test
def test_watertight_quad_shared_edge_and_exact_t(oracle_lib):
    L = oracle_lib.lib()
    # unit quad at z = 5 split along its diagonal
    t1 = np.array([0, 0, 5, 1, 0, 5, 1, 1, 5], np.float32)
    t2 = np.array([0, 0, 5, 1, 1, 5, 0, 1, 5], np.float32)
    rd = np.array([0, 0, 1], np.float32)
    out = np.zeros(4, np.float32)
    for s in np.linspace(0.0, 1.0, 33, dtype=np.float32):
        ro = np.array([s, s, 0], np.float32)  # exactly on the shared diagonal
        h1 = L.orc_triangle_intersect(fp(t1), fp(ro), fp(rd), np.float32(1e30), fp(out))
        h2 = L.orc_triangle_intersect(fp(t2), fp(ro), fp(rd), np.float32(1e30), fp(out))
        assert h1 or h2, "watertight: a ray through the shared edge must hit one of the triangles"
    rng = np.random.default_rng(1)
    for _ in range(200):
        x, y = rng.random(2).astype(np.float32)
        ro = np.array([x, y, 0], np.float32)
        h = L.orc_triangle_intersect(fp(t1 if x > y else t2), fp(ro), fp(rd), np.float32(1e30), fp(out))
        assert h and abs(float(out[3]) - 5.0) <= 2 * float(np.spacing(np.float32(5.0)))  # analytic t, <= 2 ulp
        assert abs(out[0] + out[1] + out[2] - 1) < 1e-6
    # tMax excludes farther hits; a ray pointing away misses
    ro = np.array([0.7, 0.2, 0], np.float32)
    assert not L.orc_triangle_intersect(fp(t1), fp(ro), fp(rd), np.float32(4.0), fp(out))
    assert not L.orc_triangle_intersect(fp(t1), fp(ro), fp(-rd), np.float32(1e30), fp(out))


# -------------------------------------------------------------------------------- (10) Möller overlap
def test_moller_truth_table(oracle_lib):
    L = oracle_lib.lib()
    c = np.zeros(3, np.float32)
    h = np.ones(3, np.float32)
    cases = [
        ([-0.5, -0.5, 0, 0.5, -0.5, 0, 0, 0.5, 0], True),      # inside
        ([5, 5, 5, 6, 5, 5, 5, 6, 5], False),                   # far outside
        ([1, -0.5, -0.5, 1, 0.5, -0.5, 1, 0, 0.5], True),        # lying on the +x face
        ([1.01, -0.5, -0.5, 1.01, 0.5, -0.5, 1.01, 0, 0.5], False),  # just outside the +x face
        ([-3, 0, 0, 3, 0.1, 0, 0, 3, 0.2], True),              # large triangle cutting through the box
        ([-3, -3, 0.5, 3, -3, 0.5, -3, 3, 0.5], True),         # box corner region under a big triangle
        ([2, 2, -5, 2, 2, 5, 3, 3, 0], False),                 # diagonal sliver outside the box edge
    ]
    for tri, want in cases:
        t = np.array(tri, np.float32)
        assert bool(L.orc_tribox_overlap(fp(c), fp(h), fp(t))) == want, tri


# ------------------------------------------------------------------------------------- (11) camera
def test_camera_centre_ray_and_thin_lens_focus(oracle_lib):
    L = oracle_lib.lib()
    cam = scene.PerspectiveCamera(res=(500, 500), lens_radius=0.0, focal_distance=800.0)
    d = cam.desc()
    smp = capi.rt_sampler_desc(capi.RT_SAMPLER_INDEPENDENT, 16, 1, 0, 0)
    ro, rd = np.zeros(3, np.float32), np.zeros(3, np.float32)
    L.orc_camera_ray(C.byref(d), C.byref(smp), 250, 250, 0, 250.0, 250.0, fp(ro), fp(rd))
    assert np.allclose(rd, [0, 0, 1], atol=1e-6) and np.allclose(ro, 0)
    # thin lens: rays through one raster point with different lens samples meet at z = focal_distance
    cam = scene.PerspectiveCamera(res=(500, 500), lens_radius=50.0, focal_distance=800.0)
    d = cam.desc()
    pts = []
    for idx in range(8):
        L.orc_camera_ray(C.byref(d), C.byref(smp), 10, 20, idx, 123.25, 321.75, fp(ro), fp(rd))
        t = (800.0 - ro[2]) / rd[2]
        pts.append(ro + t * rd)
        assert abs(float(np.hypot(ro[0], ro[1]))) <= 50.0 + 1e-3
    pts = np.array(pts)
    assert np.ptp(pts[:, 0]) < 1e-2 and np.ptp(pts[:, 1]) < 1e-2


# -------------------------------------------------------------------- (12) Monte Carlo known answer
def test_monte_carlo_integral_known_answer(oracle_lib):
    """MonteCarlosTestApp.h:67-68: integral_5^12 (cos x + 5) dx = 35.4223513567, estimated with the
    oracle's stratified 1-D sampler (uniform estimator, MonteCarlos.h:120-214)."""
    L = oracle_lib.lib()
    d = capi.rt_sampler_desc(capi.RT_SAMPLER_STRATIFIED, 64, 64, 1, 0)
    ops = (C.c_int * 1)(1)
    acc = 0.0
    n = 4096
    for idx in range(n):
        out = (C.c_float * 1)()
        L.orc_sampler_draws(C.byref(d), 1, 1, idx, 1, ops, out)
        x = 5 + 7 * out[0]
        acc += (math.cos(x) + 5) * 7
    assert abs(acc / n - 35.4223513567) < 1e-3
