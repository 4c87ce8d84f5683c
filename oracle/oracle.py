"""ctypes loader for the oracle (oracle/_build/librtcore.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the checker) and the
cpu_baseline leg of bench.py.  The product package never imports this module.
"""
import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB = ORACLE_DIR / "_build" / "librtcore.so"


def build(quiet=True):
    r = subprocess.run(["make", "-C", str(ORACLE_DIR)], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)
    return LIB


def use_native():
    """bench.py's cpu_baseline leg: rebuild the restatement with -O3 -march=native for the host it runs on (SURVEY
    §8d; ~5 s of g++ on the GPU box's own CPU, so the binary matches that CPU) and load it instead of the -O2
    parity build.  -ffp-contract=off and no fast-math either way, so both builds compute the same bits."""
    global LIB
    if _lib is not None:
        raise RuntimeError("oracle library already loaded")
    out = ORACLE_DIR / "_build" / "librtcore_native.so"
    r = subprocess.run(["make", "-C", str(ORACLE_DIR), "native", "-B"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle native build failed:\n" + r.stdout + r.stderr)
    LIB = out
    return out


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        from computational_ray_tracer_amd import capi
        L = C.CDLL(str(LIB))
        P = C.POINTER
        sig = {
            "orc_murmur64a": ([P(C.c_uint8), C.c_uint64, C.c_uint64], C.c_uint64),
            "orc_mixbits": ([C.c_uint64], C.c_uint64),
            "orc_hash_pixel": ([C.c_int, C.c_int, C.c_int], C.c_uint64),
            "orc_hash_pixel_dim": ([C.c_int, C.c_int, C.c_int, C.c_int], C.c_uint64),
            "orc_permutation_element": ([C.c_uint32, C.c_uint32, C.c_uint32], C.c_int),
            "orc_pcg_draws": ([C.c_int, C.c_uint64, C.c_int64, C.c_int, P(C.c_uint32)], None),
            "orc_sampler_draws": ([P(capi.rt_sampler_desc), C.c_int, C.c_int, C.c_int, C.c_int, P(C.c_int), P(C.c_float)], C.c_int),
            "orc_sample_visible": ([C.c_float, P(C.c_float), P(C.c_float)], None),
            "orc_sampler_draws_res": ([P(capi.rt_sampler_desc), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       P(C.c_int), P(C.c_float)], C.c_int),
            "orc_sobol_index": ([C.c_int] * 5, C.c_int64),
            "orc_sobol_sample": ([C.c_int64, C.c_int, C.c_int, C.c_uint32, C.c_int], C.c_float),
            "orc_visible_pdf": ([C.c_float], C.c_float),
            "orc_sample_visible_wavelength": ([C.c_float], C.c_float),
            "orc_disk_concentric": ([C.c_float, C.c_float, P(C.c_float)], None),
            "orc_sample_tent": ([C.c_float, C.c_float], C.c_float),
            "orc_spectra_dense": ([P(C.c_float)] * 4, None),
            "orc_spectra_query": ([C.c_int, C.c_int, P(C.c_float), P(C.c_float)], None),
            "orc_inner_product_y_d65": ([], C.c_float),
            "orc_sigmoid_eval": ([C.c_float] * 4, C.c_float),
            "orc_fr_dielectric": ([C.c_float, C.c_float], C.c_float),
            "orc_refract": ([P(C.c_float), P(C.c_float), C.c_float, P(C.c_float)], C.c_int),
            "orc_bk7_eta": ([C.c_float], C.c_float),
            "orc_power_heuristic": ([C.c_float, C.c_float], C.c_float),
            "orc_triangle_intersect": ([P(C.c_float), P(C.c_float), P(C.c_float), C.c_float, P(C.c_float)], C.c_int),
            "orc_tribox_overlap": ([P(C.c_float)] * 3, C.c_int),
            "orc_bounds_intersect": ([P(C.c_float), P(C.c_float), P(C.c_float), C.c_float], C.c_int),
            "orc_camera_ray": ([P(capi.rt_camera_desc), P(capi.rt_sampler_desc), C.c_int, C.c_int, C.c_int, C.c_float,
                                C.c_float, P(C.c_float), P(C.c_float)], None),
            "orc_filter_sample": ([P(capi.rt_film_desc), C.c_float, C.c_float, P(C.c_float)], None),
            "orc_scene_create": ([P(capi.rt_scene_desc), P(capi.rt_camera_desc), P(capi.rt_sampler_desc),
                                  P(capi.rt_film_desc), P(capi.rt_integrator_desc)], C.c_void_p),
            "orc_scene_destroy": ([C.c_void_p], None),
            "orc_octree_info": ([C.c_void_p, P(C.c_int), P(C.c_int), P(C.c_int)], C.c_int),
            "orc_octree_export": ([C.c_void_p, P(C.c_float), P(C.c_int), P(C.c_int), P(C.c_int), P(C.c_int)], C.c_int),
            "orc_backface_flags": ([C.c_void_p, P(C.c_uint8)], C.c_int),
            "orc_trace": ([C.c_void_p, C.c_int, P(C.c_float), P(C.c_float), C.c_int, P(C.c_int), P(C.c_float), P(C.c_int64)], C.c_int),
            "orc_occluded": ([C.c_void_p, C.c_int, P(C.c_float), P(C.c_float), P(C.c_float), P(C.c_int)], C.c_int),
            "orc_samples": ([C.c_void_p, C.c_int, P(C.c_int), P(C.c_int), P(capi.rt_sample_record)], C.c_int),
            "orc_rgb_table_lookup": ([P(C.c_float), P(C.c_float), C.c_int, C.c_int, P(C.c_float), P(C.c_float)],
                                     C.c_int),
            "orc_canonical_check": ([C.c_void_p, C.c_int, P(C.c_float), P(C.c_float), P(C.c_float), C.c_int, C.c_int,
                                     P(C.c_int64)], C.c_int),
            "orc_bvh_check": ([C.c_void_p, P(C.c_float), C.c_int, P(C.c_float), C.c_int, P(C.c_float), C.c_int,
                               P(C.c_float), C.c_int, P(C.c_float), C.c_int,
                               P(C.c_float), P(C.c_float), P(C.c_float), C.c_int, C.c_int, P(C.c_int64)], C.c_int),
            "orc_bvh_query": ([C.c_void_p, P(C.c_float), C.c_int, P(C.c_float), C.c_int, P(C.c_float), C.c_int,
                               P(C.c_float), C.c_int, P(C.c_float), C.c_int,
                               P(C.c_float), P(C.c_float), P(C.c_float), C.c_int, C.c_int, P(C.c_int), P(C.c_float),
                               P(C.c_int), P(C.c_int)], C.c_int),
            "orc_render": ([C.c_void_p, C.c_int, C.c_int, P(C.c_float), C.c_int, P(C.c_int64), P(C.c_int), C.c_int], C.c_int),
            "orc_resolve": ([C.c_void_p, P(C.c_float), P(C.c_uint8)], None),
            "orc_resolve_srgb": ([C.c_void_p, P(C.c_float), P(C.c_uint8)], None),
            "orc_resolve_matrices": ([C.c_void_p, P(C.c_float), P(C.c_float)], None),
            "orc_sensor_training": ([C.c_void_p, P(C.c_float), P(C.c_float)], None),
        }
        for name, (a, r) in sig.items():
            f = getattr(L, name)
            f.argtypes = a
            f.restype = r
        _lib = L
    return _lib


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def iptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


class OracleScene:
    """Oracle twin of a product context, built from the same descriptors (a scene.Config)."""

    def __init__(self, cfg):
        self.cfg = cfg
        L = lib()
        self._sd = cfg.model.desc()
        self._cd = cfg.camera.desc()
        self._smp = cfg.sampler.desc()
        self._fd = cfg.film.desc()
        self._id = cfg.integrator.desc()
        self.h = L.orc_scene_create(C.byref(self._sd), C.byref(self._cd), C.byref(self._smp), C.byref(self._fd),
                                    C.byref(self._id))
        self.res = cfg.film.res

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_scene_destroy(self.h)
            self.h = None

    def octree(self):
        L = lib()
        n, r, d = C.c_int(), C.c_int(), C.c_int()
        L.orc_octree_info(self.h, C.byref(n), C.byref(r), C.byref(d))
        b = np.zeros((n.value, 6), np.float32)
        ch = np.zeros(n.value, np.int32)
        lf = np.zeros(n.value, np.int32)
        lc = np.zeros(n.value, np.int32)
        refs = np.zeros(max(r.value, 1), np.int32)
        rc = L.orc_octree_export(self.h, fptr(b), iptr(ch), iptr(lf), iptr(lc), iptr(refs))
        assert rc == 0, "octree children not contiguous"
        return dict(bounds=b, child=ch, leaf_first=lf, leaf_count=lc, refs=refs[: r.value], depth=d.value)

    def backface_flags(self):
        out = np.zeros(len(self.cfg.model.indices), np.uint8)
        lib().orc_backface_flags(self.h, out.ctypes.data_as(C.POINTER(C.c_uint8)))
        return out

    def trace(self, ro, rd, use_cull=True):
        ro = np.ascontiguousarray(ro, np.float32)
        rd = np.ascontiguousarray(rd, np.float32)
        n = len(ro)
        prim = np.zeros(n, np.int32)
        bt = np.zeros((n, 4), np.float32)
        cnt = np.zeros(2, np.int64)
        lib().orc_trace(self.h, n, fptr(ro), fptr(rd), int(use_cull), iptr(prim), fptr(bt),
                        cnt.ctypes.data_as(C.POINTER(C.c_int64)))
        return prim, bt, cnt

    def occluded(self, ro, rd, tmax):
        ro = np.ascontiguousarray(ro, np.float32)
        rd = np.ascontiguousarray(rd, np.float32)
        tmax = np.ascontiguousarray(tmax, np.float32)
        occ = np.zeros(len(ro), np.int32)
        lib().orc_occluded(self.h, len(ro), fptr(ro), fptr(rd), fptr(tmax), iptr(occ))
        return occ

    def canonical_check(self, ro, rd, tmax, use_cull=False, nthreads=None):
        """Canonical fast-path rule vs the reference BFS on every ray; returns a dict of counts."""
        ro = np.ascontiguousarray(ro, np.float32)
        rd = np.ascontiguousarray(rd, np.float32)
        tmax = np.ascontiguousarray(tmax, np.float32)
        st = np.zeros(8, np.int64)
        lib().orc_canonical_check(self.h, len(ro), fptr(ro), fptr(rd), fptr(tmax), int(use_cull),
                                  nthreads or (os.cpu_count() or 1), st.ctypes.data_as(C.POINTER(C.c_int64)))
        keys = ["closest_mismatch", "closest_ambiguous", "anyhit_mismatch", "anyhit_ambiguous", "hits", "occluded",
                "rays", "first_mismatch"]
        return dict(zip(keys, (int(x) for x in st)))

    def bvh_check(self, bvh, ro, rd, tmax, use_cull=False, nthreads=None, bvh_any=None):
        """The GPU's walk restated (Bvh8) over the product-built BVH `bvh` (dict: nodes (n, 32) f32, tiles (m, 12)
        f32, consts (wabs, oguard)) against the reference BFS on every ray; returns counts.
        `bvh_any`: tile set 0's BVH for the any-hit queries when `bvh` is the culled set's (default: `bvh`)."""
        ro = np.ascontiguousarray(ro, np.float32)
        rd = np.ascontiguousarray(rd, np.float32)
        tmax = np.ascontiguousarray(tmax, np.float32)
        nd, tl, cs = (np.ascontiguousarray(bvh[k], np.float32) for k in ("nodes", "tiles", "consts"))
        ba = bvh_any or bvh
        nda, tla = (np.ascontiguousarray(ba[k], np.float32) for k in ("nodes", "tiles"))
        st = np.zeros(16, np.int64)
        lib().orc_bvh_check(self.h, fptr(nd), len(nd), fptr(tl), len(tl), fptr(nda), len(nda), fptr(tla), len(tla),
                            fptr(cs), len(ro), fptr(ro), fptr(rd),
                            fptr(tmax), int(use_cull), nthreads or (os.cpu_count() or 1),
                            st.ctypes.data_as(C.POINTER(C.c_int64)))
        keys = ["closest_mismatch", "closest_ambiguous", "anyhit_mismatch", "anyhit_ambiguous", "hits", "occluded",
                "rays", "first_mismatch", "closest_nodes", "closest_boxes", "closest_tris", "max_stack",
                "anyhit_nodes", "anyhit_boxes", "anyhit_tris", "stack_overflows"]
        return dict(zip(keys, (int(x) for x in st)))

    def bvh_query(self, bvh, ro, rd, tmax=None, use_cull=False, nthreads=None, bvh_any=None):
        """Per ray, what the GPU must return over `bvh`: the canonical closest hit / any hit of the restated walk, the
        reference BFS's for ambiguous rays.  Returns (prim, bt, occluded, amb)."""
        ro = np.ascontiguousarray(ro, np.float32)
        rd = np.ascontiguousarray(rd, np.float32)
        n = len(ro)
        nd, tl, cs = (np.ascontiguousarray(bvh[k], np.float32) for k in ("nodes", "tiles", "consts"))
        ba = bvh_any or bvh
        nda, tla = (np.ascontiguousarray(ba[k], np.float32) for k in ("nodes", "tiles"))
        prim = np.zeros(n, np.int32)
        bt = np.zeros((n, 4), np.float32)
        occ = np.zeros(n, np.int32)
        amb = np.zeros(n, np.int32)
        tm = None if tmax is None else np.ascontiguousarray(tmax, np.float32)
        lib().orc_bvh_query(self.h, fptr(nd), len(nd), fptr(tl), len(tl), fptr(nda), len(nda), fptr(tla), len(tla),
                            fptr(cs), n, fptr(ro), fptr(rd),
                            fptr(tm) if tm is not None else None, int(use_cull), nthreads or (os.cpu_count() or 1),
                            iptr(prim), fptr(bt), iptr(occ), iptr(amb))
        return prim, bt, occ, amb

    def samples(self, pixel_ids, indices):
        from computational_ray_tracer_amd import capi
        pixel_ids = np.ascontiguousarray(pixel_ids, np.int32)
        indices = np.ascontiguousarray(indices, np.int32)
        out = (capi.rt_sample_record * len(pixel_ids))()
        lib().orc_samples(self.h, len(pixel_ids), iptr(pixel_ids), iptr(indices), out)
        return out

    def render(self, index_begin, index_end, film=None, nthreads=None, pixel_ids=None):
        if film is None:
            film = np.zeros((self.res[0] * self.res[1], 4), np.float32)
        if nthreads is None:
            nthreads = min(os.cpu_count() or 1, 16)  # tests; bench.py's baseline passes os.cpu_count()
        cnt = np.zeros(5, np.int64)
        if pixel_ids is not None:
            pixel_ids = np.ascontiguousarray(pixel_ids, np.int32)
            pp, npx = iptr(pixel_ids), len(pixel_ids)
        else:
            pp, npx = None, 0
        lib().orc_render(self.h, index_begin, index_end, fptr(film), nthreads, cnt.ctypes.data_as(C.POINTER(C.c_int64)),
                         pp, npx)
        self.counters = cnt
        return film

    def resolve_matrices(self):
        """(XYZFromSensorRGB, RGBFromXYZ) as column-major float32[9] (glm layout)."""
        a, b = np.zeros(9, np.float32), np.zeros(9, np.float32)
        lib().orc_resolve_matrices(self.h, fptr(a), fptr(b))
        return a, b

    def sensor_training(self):
        """Camera sensors: the 24 swatches' (camera RGB, target XYZ) rows of the least-squares fit."""
        a, b = np.zeros((24, 3), np.float32), np.zeros((24, 3), np.float32)
        lib().orc_sensor_training(self.h, fptr(a), fptr(b))
        return a, b

    def resolve(self, film, srgb=False):
        out = np.zeros((self.res[0] * self.res[1], 3), np.uint8)
        f = lib().orc_resolve_srgb if srgb else lib().orc_resolve
        f(self.h, fptr(np.ascontiguousarray(film, np.float32)), out.ctypes.data_as(C.POINTER(C.c_uint8)))
        return out
