"""Python host mirror of the reference's render loop (RayTracerTestApp::MainLoop, RayTracerTestApp.h:64-513)
driving the MI355X C-ABI.  `Renderer.render_pass(index_begin, index_end, film)` is the drop-in for one
ThreadFunction/evaluate_pixel dispatch over every pixel (RayTracerTestApp.h:347-422)."""
import ctypes as C

import numpy as np

from . import capi


class Renderer:
    """One rt_ctx.  `device` is one HIP ordinal or a list of them (rt_options.devices: every pass renders on
    all of them at once, pixel tiles interleaved, the film bit-identical to one device).  Configured from a
    scene.Config (or the individual descriptors)."""

    def __init__(self, cfg=None, device=0, octree_build=capi.RT_OCTREE_BUILD_DEVICE):
        self.lib = capi.load_library()
        opt = capi.rt_options()
        devs = list(device) if isinstance(device, (list, tuple)) else [int(device)]
        if not 1 <= len(devs) <= capi.RT_MAX_DEVICES:
            raise ValueError(f"1..{capi.RT_MAX_DEVICES} devices")
        opt.device = devs[0]
        opt.n_devices = len(devs)
        for i, d in enumerate(devs):
            opt.devices[i] = d
        opt.octree_build = octree_build
        h = C.c_void_p()
        rc = self.lib.rt_create(C.byref(opt), C.byref(h))
        if rc != capi.RT_OK:
            raise capi.RTError("rt_create", rc, "no usable gfx950 device" if rc == capi.RT_E_NODEVICE else "")
        self.h = h
        self.cfg = None
        if cfg is not None:
            self.configure(cfg)

    def _chk(self, name, rc):
        if rc != capi.RT_OK:
            raise capi.RTError(name, rc, self.lib.rt_last_error(self.h).decode())

    def configure(self, cfg):
        self.cfg = cfg
        self._scene = cfg.model.desc()
        self._chk("rt_scene_upload", self.lib.rt_scene_upload(self.h, C.byref(self._scene)))
        self._chk("rt_camera_set", self.lib.rt_camera_set(self.h, C.byref(cfg.camera.desc())))
        self._chk("rt_sampler_set", self.lib.rt_sampler_set(self.h, C.byref(cfg.sampler.desc())))
        self._chk("rt_film_set", self.lib.rt_film_set(self.h, C.byref(cfg.film.desc())))
        self._chk("rt_integrator_set", self.lib.rt_integrator_set(self.h, C.byref(cfg.integrator.desc())))
        self.res = cfg.film.res

    def set_shard(self, tile_size, n_shards, shard_id):
        self._chk("rt_set_shard", self.lib.rt_set_shard(self.h, tile_size, n_shards, shard_id))

    def new_film(self):
        return np.zeros((self.res[0] * self.res[1], 4), dtype=np.float32)

    def render_pass(self, index_begin, index_end, film=None):
        """Accumulate sample indices [index_begin, index_end) into `film` (host float32 [W*H, 4])."""
        if film is None:
            film = self.new_film()
        assert film.dtype == np.float32 and film.flags.c_contiguous and film.shape == (self.res[0] * self.res[1], 4)
        self._chk("rt_render_pass", self.lib.rt_render_pass(self.h, index_begin, index_end,
                                                            film.ctypes.data_as(C.POINTER(capi.rt_pixel))))
        return film

    def render_pass_device(self, index_begin, index_end, film_ptr, stream_ptr=None):
        """Accumulate into a device-resident film (e.g. a torch.cuda float32 [W*H, 4] tensor's data_ptr)."""
        self._chk("rt_render_pass_device", self.lib.rt_render_pass_device(
            self.h, index_begin, index_end, C.c_void_p(film_ptr), C.c_void_p(stream_ptr or 0)))

    def resolve(self, film, srgb=False):
        """rt_film_resolve (the reference's linear 255·x) or rt_film_resolve_srgb (pbrt's sRGB encoding)."""
        out = np.zeros((self.res[0] * self.res[1], 3), np.uint8)
        name = "rt_film_resolve_srgb" if srgb else "rt_film_resolve"
        self._chk(name, getattr(self.lib, name)(self.h, np.ascontiguousarray(film, np.float32).ctypes.data_as(
            C.POINTER(capi.rt_pixel)), out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out

    def film_matrices(self):
        """(XYZFromSensorRGB, RGBFromXYZ) of the current film's sensor, column-major float32[9] each."""
        a, b = np.zeros(9, np.float32), np.zeros(9, np.float32)
        P = lambda x: x.ctypes.data_as(C.POINTER(C.c_float))
        self._chk("rt_film_matrices", self.lib.rt_film_matrices(self.h, P(a), P(b)))
        return a, b

    def stats(self):
        s = capi.rt_stats()
        self._chk("rt_get_stats", self.lib.rt_get_stats(self.h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in s._fields_}

    def reset_stats(self):
        self._chk("rt_reset_stats", self.lib.rt_reset_stats(self.h))

    def octree(self):
        info = capi.rt_octree_info()
        self._chk("rt_octree_get_info", self.lib.rt_octree_get_info(self.h, C.byref(info)))
        n, r = info.n_nodes, info.n_leaf_refs
        b = np.zeros((n, 6), np.float32)
        ch, lf, lc = (np.zeros(n, np.int32) for _ in range(3))
        refs = np.zeros(max(r, 1), np.int32)
        P = lambda a, t: a.ctypes.data_as(C.POINTER(t))
        self._chk("rt_octree_export", self.lib.rt_octree_export(self.h, P(b, C.c_float), P(ch, C.c_int32), P(lf, C.c_int32),
                                                                P(lc, C.c_int32), P(refs, C.c_int32)))
        return dict(bounds=b, child=ch, leaf_first=lf, leaf_count=lc, refs=refs[:r], depth=info.depth,
                    max_queue_groups=info.max_queue_groups)

    def bvh(self, tile_set=0):
        """The fast traversal's BVH as uploaded (rt_bvh_export): nodes (n, 32) f32, tiles (m, 12) f32, consts."""
        return _bvh_arrays(lambda nn, nt, cs, nd, tl: self.lib.rt_bvh_export(self.h, tile_set, nn, nt, cs, nd, tl),
                           lambda rc: self._chk("rt_bvh_export", rc))

    def trace(self, ro, rd, use_cull=True):
        ro = np.ascontiguousarray(ro, np.float32)
        rd = np.ascontiguousarray(rd, np.float32)
        n = len(ro)
        prim = np.zeros(n, np.int32)
        bt = np.zeros((n, 4), np.float32)
        P = lambda a, t: a.ctypes.data_as(C.POINTER(t))
        self._chk("rt_debug_trace", self.lib.rt_debug_trace(self.h, n, P(ro, C.c_float), P(rd, C.c_float), int(use_cull),
                                                            P(prim, C.c_int32), P(bt, C.c_float)))
        return prim, bt

    def occluded(self, ro, rd, tmax):
        """Shadow query of the path kernels (any hit within tmax): int32 0/1 per ray."""
        ro = np.ascontiguousarray(ro, np.float32)
        rd = np.ascontiguousarray(rd, np.float32)
        tmax = np.ascontiguousarray(tmax, np.float32)
        occ = np.zeros(len(ro), np.int32)
        P = lambda a, t: a.ctypes.data_as(C.POINTER(t))
        self._chk("rt_debug_occluded", self.lib.rt_debug_occluded(self.h, len(ro), P(ro, C.c_float), P(rd, C.c_float),
                                                                  P(tmax, C.c_float), P(occ, C.c_int32)))
        return occ

    def debug_sort(self, which, S, shard_len, keys, slots=None, bits_a=3, bits_b=3):
        """rt_debug_sort: the ray (which 0) or NEE (which 1) coherence sort on a synthetic sharded queue; returns the
        output array (8 S int32: queue positions / slots at the sorted positions) and the rewritten shard lengths."""
        shard_len = np.ascontiguousarray(shard_len, np.int32)
        keys = np.ascontiguousarray(keys, np.uint32)
        assert len(shard_len) == capi.QUEUE_SHARDS and len(keys) == capi.QUEUE_SHARDS * S
        sl = None if slots is None else np.ascontiguousarray(slots, np.int32)
        out = np.zeros(capi.QUEUE_SHARDS * S, np.int32)
        olen = np.zeros(capi.QUEUE_SHARDS, np.int32)
        P = lambda a, t: a.ctypes.data_as(C.POINTER(t))
        self._chk("rt_debug_sort", self.lib.rt_debug_sort(self.h, int(which), int(S), P(shard_len, C.c_int32),
                                                          P(keys, C.c_uint32), None if sl is None else P(sl, C.c_int32),
                                                          int(bits_a), int(bits_b), P(out, C.c_int32),
                                                          P(olen, C.c_int32)))
        return out, olen

    def samples(self, pixel_ids, indices):
        pixel_ids = np.ascontiguousarray(pixel_ids, np.int32)
        indices = np.ascontiguousarray(indices, np.int32)
        out = (capi.rt_sample_record * len(pixel_ids))()
        P = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))
        self._chk("rt_debug_samples", self.lib.rt_debug_samples(self.h, len(pixel_ids), P(pixel_ids), P(indices), out))
        return out

    def close(self):
        if getattr(self, "h", None):
            self.lib.rt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def records_to_arrays(recs):
    """rt_sample_record array -> dict of numpy arrays (for bit-exact comparisons)."""
    raw = np.frombuffer(bytes(recs), dtype=np.float32).reshape(len(recs), 39)
    return dict(lam=raw[:, 0:8], pdf=raw[:, 8:16], ro=raw[:, 16:19], rd=raw[:, 19:22],
                prim=raw[:, 22].view(np.int32), b=raw[:, 23:26], t=raw[:, 26], L=raw[:, 27:35], rgb=raw[:, 35:38],
                weight=raw[:, 38])


def _bvh_arrays(call, check):
    P = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
    nn, nt = C.c_int(), C.c_int()
    cs = np.zeros(2, np.float32)
    check(call(C.byref(nn), C.byref(nt), P(cs), None, None))
    nodes = np.zeros((max(nn.value, 1), 32), np.float32)
    tiles = np.zeros((max(nt.value, 1), 12), np.float32)
    check(call(C.byref(nn), C.byref(nt), P(cs), P(nodes), P(tiles)))
    return dict(nodes=nodes[: nn.value], tiles=tiles[: nt.value], consts=cs)


def build_bvh_host(model, tile_set=0):
    """rt_debug_bvh_build: the upload's BVH built on the host from a scene.Model, without a device (CPU tests)."""
    lib = capi.load_library()
    sd = model.desc()

    def check(rc):
        if rc != capi.RT_OK:
            raise capi.RTError("rt_debug_bvh_build", rc, "bad scene")
    return _bvh_arrays(lambda nn, nt, cs, nd, tl: lib.rt_debug_bvh_build(C.byref(sd), tile_set, nn, nt, cs, nd, tl),
                       check)
