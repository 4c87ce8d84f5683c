"""ctypes mirror of include/rtmi355x.h (the drop-in C-ABI) and the loader of librtmi355x.so.

The shared library is built in-tree (computational_ray_tracer_amd/lib/librtmi355x.so) by
`python __graft_entry__.py build` / `make -C computational_ray_tracer_amd/csrc`.  Loading fails
loudly when it is missing: there is no Python or CPU fallback for the hot path.
"""
import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "lib" / "librtmi355x.so"

RT_OK, RT_E_ARG, RT_E_HIP, RT_E_RCCL, RT_E_OOM, RT_E_STATE, RT_E_NODEVICE, RT_E_LIMIT = 0, -1, -2, -3, -4, -5, -6, -7
STATUS_NAMES = {0: "RT_OK", -1: "RT_E_ARG", -2: "RT_E_HIP", -3: "RT_E_RCCL", -4: "RT_E_OOM", -5: "RT_E_STATE",
                -6: "RT_E_NODEVICE", -7: "RT_E_LIMIT"}
RT_MAT_DIFFUSE, RT_MAT_MIRROR, RT_MAT_DIELECTRIC = 0, 1, 2
RT_SHAPE_SPHERE, RT_SHAPE_DISK, RT_SHAPE_TRIANGLE = 0, 1, 2
RT_LIGHT_QUAD, RT_LIGHT_DISK, RT_LIGHT_POINT, RT_LIGHT_DISTANT = 0, 1, 2, 3
RT_CAMERA_PERSPECTIVE, RT_CAMERA_ORTHOGRAPHIC, RT_CAMERA_PINHOLE, RT_CAMERA_THINLENS = 0, 1, 2, 3
RT_SAMPLER_INDEPENDENT, RT_SAMPLER_STRATIFIED, RT_SAMPLER_SOBOL = 0, 1, 2
RT_SOBOL_NONE, RT_SOBOL_PERMUTE_DIGITS, RT_SOBOL_FAST_OWEN, RT_SOBOL_OWEN = 0, 1, 2, 3
RT_FILTER_BOX, RT_FILTER_TRIANGLE, RT_FILTER_GAUSSIAN, RT_FILTER_LANCZOS = 0, 1, 2, 3
RT_SENSOR_XYZ, RT_SENSOR_CANON_EOS_100D, RT_SENSOR_COUNT = 0, 1, 18
RT_OCTREE_BUILD_DEVICE, RT_OCTREE_BUILD_HOST = 0, 1
RT_ILLUM_D65, RT_ILLUM_A, RT_ILLUM_D50, RT_ILLUM_F1, RT_ILLUM_ACES_D60, RT_ILLUM_COUNT = 0, 1, 2, 3, 15, 16
RT_INTEGRATOR_REFERENCE, RT_INTEGRATOR_PATH, RT_INTEGRATOR_PATH_MIS = 0, 1, 2
ABI_VERSION = 9
RT_MAX_DEVICES = 16
QUEUE_SHARDS = 8  # RT_QUEUE_SHARDS

F16 = C.c_float * 16
F9 = C.c_float * 9
F3 = C.c_float * 3
F2 = C.c_float * 2
F8 = C.c_float * 8


class rt_options(C.Structure):
    _fields_ = [("device", C.c_int), ("octree_build", C.c_int), ("n_devices", C.c_int),
                ("devices", C.c_int * RT_MAX_DEVICES), ("reserved", C.c_int * 5)]


class rt_pixel(C.Structure):
    _fields_ = [("r", C.c_float), ("g", C.c_float), ("b", C.c_float), ("w", C.c_float)]


class rt_material(C.Structure):
    _fields_ = [("type", C.c_int), ("sigmoid", F3), ("emission_scale", C.c_float), ("eta", C.c_float)]


class rt_shape(C.Structure):
    _fields_ = [("type", C.c_int), ("object_to_render", F16), ("render_to_object", F16), ("normal_to_render", F9),
                ("radius", C.c_float), ("zmin", C.c_float), ("zmax", C.c_float), ("phimax", C.c_float),
                ("height", C.c_float), ("inner_radius", C.c_float), ("outer_radius", C.c_float),
                ("p", F9), ("material", C.c_int)]


class rt_light(C.Structure):
    _fields_ = [("type", C.c_int), ("p", F3), ("e1", F3), ("e2", F3), ("n", F3), ("dir", F3), ("scale", C.c_float),
                ("shape", C.c_int), ("material", C.c_int)]


class rt_scene_desc(C.Structure):
    _fields_ = [
        ("n_vertices", C.c_int), ("positions", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
        ("n_triangles", C.c_int), ("indices", C.POINTER(C.c_uint32)),
        ("object_to_render", F16), ("normal_to_render", F9),
        ("cull_backfaces", C.c_int), ("cull_look", F3), ("octree_capacity", C.c_int),
        ("tri_material", C.POINTER(C.c_int32)),
        ("n_materials", C.c_int), ("materials", C.POINTER(rt_material)),
        ("n_lights", C.c_int), ("lights", C.POINTER(rt_light)),
        ("n_shapes", C.c_int), ("shapes", C.POINTER(rt_shape)),
    ]


class rt_camera_desc(C.Structure):
    _fields_ = [("type", C.c_int), ("raster_to_camera", F16), ("camera_to_world", F16),
                ("lens_radius", C.c_float), ("focal_distance", C.c_float), ("raster_to_screen", F16),
                ("pinhole_depth", C.c_float), ("thin_focal", C.c_float), ("thin_aperture_diameter", C.c_float),
                ("sensor_depth", C.c_float)]


class rt_sampler_desc(C.Structure):
    _fields_ = [("kind", C.c_int), ("x_samples", C.c_int), ("y_samples", C.c_int), ("jitter", C.c_int),
                ("seed", C.c_int), ("randomize", C.c_int)]


class rt_film_desc(C.Structure):
    _fields_ = [("res_x", C.c_int), ("res_y", C.c_int), ("filter", C.c_int), ("filter_radius", F2),
                ("imaging_ratio", C.c_float), ("filter_param", C.c_float), ("sensor", C.c_int),
                ("sensor_illum", C.c_int)]


class rt_integrator_desc(C.Structure):
    _fields_ = [("kind", C.c_int), ("max_depth", C.c_int), ("albedo_rgb", F3)]


class rt_stats(C.Structure):
    _fields_ = [("samples", C.c_int64), ("rays", C.c_int64), ("shadow_rays", C.c_int64),
                ("nodes_tested", C.c_int64), ("tris_tested", C.c_int64), ("shadow_nodes_tested", C.c_int64),
                ("shadow_tris_tested", C.c_int64), ("hits", C.c_int64),
                ("ms_generate", C.c_double), ("ms_trace", C.c_double), ("ms_shade", C.c_double),
                ("ms_shadow", C.c_double), ("ms_film", C.c_double), ("launches_trace", C.c_int64),
                ("launches_shade", C.c_int64), ("fallback_rays", C.c_int64), ("shadow_fallback_rays", C.c_int64),
                ("ms_sort", C.c_double), ("nee_vertices", C.c_int64), ("coop_overflows", C.c_int64)]


class rt_sample_record(C.Structure):
    _fields_ = [("lambda_", F8), ("pdf", F8), ("ro", F3), ("rd", F3), ("prim", C.c_int32), ("b", F3),
                ("t", C.c_float), ("L", F8), ("rgb", F3), ("weight", C.c_float)]


class rt_mesh(C.Structure):
    _fields_ = [("n_vertices", C.c_int), ("positions", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("texcoords", C.POINTER(C.c_float)), ("n_triangles", C.c_int), ("indices", C.POINTER(C.c_uint32))]


class rt_octree_info(C.Structure):
    _fields_ = [("n_nodes", C.c_int), ("n_leaf_refs", C.c_int), ("max_queue_groups", C.c_int), ("depth", C.c_int),
                ("bvh_nodes", C.c_int), ("bvh_depth", C.c_int)]


# every symbol include/rtmi355x.h declares (checked by tests/test_capi_symbols.py)
EXPORTS = [
    "rt_create", "rt_destroy", "rt_last_error", "rt_abi_version",
    "rt_scene_upload", "rt_camera_set", "rt_sampler_set", "rt_film_set", "rt_integrator_set", "rt_set_shard",
    "rt_render_pass", "rt_render_pass_device", "rt_film_resolve",
    "rt_get_stats", "rt_reset_stats", "rt_octree_get_info", "rt_octree_export", "rt_bvh_export", "rt_debug_bvh_build",
    "rt_debug_trace", "rt_debug_occluded", "rt_debug_samples", "rt_debug_sort",
    "rt_film_resolve_srgb", "rt_load_obj", "rt_mesh_free", "rt_image_write", "rt_rgb_to_sigmoid", "rt_rgb_fit_sigmoid",
    "rt_sensor_name", "rt_film_matrices",
]

_lib = None


class RTError(RuntimeError):
    def __init__(self, call, status, message):
        super().__init__(f"{call} failed: {STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


def library_path():
    """The librtmi355x.so that load_library() loads (RTMI_LIB overrides the in-tree build)."""
    return Path(os.environ.get("RTMI_LIB", LIB_PATH))


def library_sha16(path=None):
    """Build id of a library file: the first 16 hex digits of its SHA-256 (profiles/counters_*.json carry the id of
    the build they were measured on; bench.py uses their PMC figures only for the same build)."""
    import hashlib
    return hashlib.sha256(Path(path or library_path()).read_bytes()).hexdigest()[:16]


def load_library(path=None):
    """Load librtmi355x.so (built in-tree).  Raises if it is missing — no fallback exists."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else library_path()  # RTMI_LIB: A/B kernel variants
    if not p.exists():
        raise RuntimeError(f"{p} is missing: build it with `python __graft_entry__.py build` "
                           "(the MI355X HIP extension is the only implementation of the hot path)")
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    P = C.POINTER
    sig = {
        "rt_create": ([P(rt_options), P(C.c_void_p)], C.c_int),
        "rt_destroy": ([C.c_void_p], None),
        "rt_last_error": ([C.c_void_p], C.c_char_p),
        "rt_abi_version": ([], C.c_int),
        "rt_scene_upload": ([C.c_void_p, P(rt_scene_desc)], C.c_int),
        "rt_camera_set": ([C.c_void_p, P(rt_camera_desc)], C.c_int),
        "rt_sampler_set": ([C.c_void_p, P(rt_sampler_desc)], C.c_int),
        "rt_film_set": ([C.c_void_p, P(rt_film_desc)], C.c_int),
        "rt_integrator_set": ([C.c_void_p, P(rt_integrator_desc)], C.c_int),
        "rt_set_shard": ([C.c_void_p, C.c_int, C.c_int, C.c_int], C.c_int),
        "rt_render_pass": ([C.c_void_p, C.c_int, C.c_int, P(rt_pixel)], C.c_int),
        "rt_render_pass_device": ([C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p], C.c_int),
        "rt_film_resolve": ([C.c_void_p, P(rt_pixel), P(C.c_uint8)], C.c_int),
        "rt_get_stats": ([C.c_void_p, P(rt_stats)], C.c_int),
        "rt_reset_stats": ([C.c_void_p], C.c_int),
        "rt_octree_get_info": ([C.c_void_p, P(rt_octree_info)], C.c_int),
        "rt_octree_export": ([C.c_void_p, P(C.c_float), P(C.c_int32), P(C.c_int32), P(C.c_int32), P(C.c_int32)], C.c_int),
        "rt_bvh_export": ([C.c_void_p, C.c_int, P(C.c_int), P(C.c_int), P(C.c_float), P(C.c_float), P(C.c_float)],
                          C.c_int),
        "rt_debug_bvh_build": ([P(rt_scene_desc), C.c_int, P(C.c_int), P(C.c_int), P(C.c_float), P(C.c_float),
                               P(C.c_float)], C.c_int),
        "rt_debug_trace": ([C.c_void_p, C.c_int, P(C.c_float), P(C.c_float), C.c_int, P(C.c_int32), P(C.c_float)], C.c_int),
        "rt_debug_occluded": ([C.c_void_p, C.c_int, P(C.c_float), P(C.c_float), P(C.c_float), P(C.c_int32)], C.c_int),
        "rt_debug_samples": ([C.c_void_p, C.c_int, P(C.c_int32), P(C.c_int32), P(rt_sample_record)], C.c_int),
        "rt_debug_sort": ([C.c_void_p, C.c_int, C.c_int, P(C.c_int32), P(C.c_uint32), P(C.c_int32), C.c_int, C.c_int,
                           P(C.c_int32), P(C.c_int32)], C.c_int),
        "rt_film_resolve_srgb": ([C.c_void_p, P(rt_pixel), P(C.c_uint8)], C.c_int),
        "rt_load_obj": ([C.c_char_p, P(P(rt_mesh))], C.c_int),
        "rt_mesh_free": ([P(rt_mesh)], None),
        "rt_image_write": ([C.c_char_p, C.c_int, C.c_int, P(C.c_uint8), C.c_int], C.c_int),
        "rt_rgb_to_sigmoid": ([P(C.c_float), P(C.c_float)], C.c_int),
        "rt_rgb_fit_sigmoid": ([P(C.c_float), P(C.c_float)], C.c_int),
        "rt_sensor_name": ([C.c_int], C.c_char_p),
        "rt_film_matrices": ([C.c_void_p, P(C.c_float), P(C.c_float)], C.c_int),
    }
    # RTMI_AB_COMPAT=1 (A/B tooling only: scripts/gpu_ab_sets.sh timing an earlier build through RTMI_LIB) accepts an
    # older ABI and skips entry points it lacks; the rt_stats fields it predates read as 0
    compat = os.environ.get("RTMI_AB_COMPAT") == "1"
    for name, (args, res) in sig.items():
        if compat and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    if lib.rt_abi_version() != ABI_VERSION and not compat:
        raise RuntimeError("librtmi355x ABI version mismatch")
    if path is None:
        _lib = lib
    return lib
