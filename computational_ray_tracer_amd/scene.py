"""Host-side scene description — the Python mirror of what RayTracerTestApp::MainLoop builds before the
render loop (Applications/RayTracerTestApp.h:70-189): meshes + TriModel transform, camera matrices,
sampler, filter, film, integrator.  Everything here produces the POD descriptors of include/rtmi355x.h;
the hot path itself lives behind the C-ABI.

Matrix math follows the reference's glm calls (Cameras.h:80-142, 253-310; Shapes.h:175-181) evaluated
in float64 and rounded once to float32 (glm is not vendored, so its float rounding is unpinned —
SURVEY.md §8c).  The same float32 matrices are handed to the HIP product and to the oracle.
"""
import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from . import capi

# ----------------------------------------------------------------------------------- glm-like helpers


def translate(v):
    m = np.eye(4)
    m[:3, 3] = v
    return m


def scale(v):
    return np.diag([v[0], v[1], v[2], 1.0])


def rotate(angle_deg, axis):
    """glm::rotate(mat4(1), radians(angle), axis)."""
    a = math.radians(angle_deg)
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.linalg.norm(axis)
    c, s = math.cos(a), math.sin(a)
    x, y, z = axis
    t = 1 - c
    r = np.array([[t * x * x + c, t * x * y - s * z, t * x * z + s * y],
                  [t * x * y + s * z, t * y * y + c, t * y * z - s * x],
                  [t * x * z - s * y, t * y * z + s * x, t * z * z + c]])
    m = np.eye(4)
    m[:3, :3] = r
    return m


PERM_YZ = np.array([[1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], dtype=np.float64)  # Shapes.h:178


def colmajor(m):
    """numpy (row, col) float64 matrix -> column-major float32 list (glm memory layout)."""
    return np.asarray(m, dtype=np.float64).T.astype(np.float32).reshape(-1)


# ----------------------------------------------------------------------------------------- camera


def _camera_base(sw, sh, res, position, look, worldup):
    """CameraBase (Cameras.h:80-142): M_RastertoScreen and M_CameratoWorld, float64."""
    rx, ry = res
    screen_to_ndc = scale((1 / sw, 1 / sh, 1)) @ translate((sw / 2, sh / 2, 0))   # Cameras.h:88-89
    ndc_to_raster = scale((rx, -ry, 1)) @ translate((0, -1, 0))                   # Cameras.h:90-91
    raster_to_screen = np.linalg.inv(ndc_to_raster @ screen_to_ndc)                # Cameras.h:93-94
    d = np.asarray(look, float)
    d = d / np.linalg.norm(d)
    r = np.cross(np.asarray(worldup, float), d)
    r = r / np.linalg.norm(r)
    u = np.cross(d, r)                                                             # Cameras.h:130-139
    cam_to_world = np.eye(4)
    cam_to_world[:3, 0], cam_to_world[:3, 1], cam_to_world[:3, 2] = r, u, d
    cam_to_world[:3, 3] = position
    return raster_to_screen, cam_to_world


def _camera_desc(kind, r2c, c2w, r2s=None, **kw):
    d = capi.rt_camera_desc()
    d.type = kind
    d.raster_to_camera[:] = colmajor(r2c).tolist()
    d.camera_to_world[:] = colmajor(c2w).tolist()
    d.raster_to_screen[:] = colmajor(r2s if r2s is not None else np.eye(4)).tolist()
    for k, v in kw.items():
        setattr(d, k, v)
    return d


@dataclass
class OrthographicCamera:
    """OrthographicCamera(near, far, sensor_w, sensor_h, pos, look, right, worldup, res) (Cameras.h:213-245)."""
    near: float = 1e-2
    far: float = 1000.0
    sensor: tuple = (500.0, 500.0)
    position: tuple = (0.0, 0.0, 0.0)
    look: tuple = (0.0, 0.0, 1.0)
    right: tuple = (1.0, 0.0, 0.0)
    worldup: tuple = (0.0, 1.0, 0.0)
    res: tuple = (500, 500)

    def desc(self):
        r2s, c2w = _camera_base(self.sensor[0], self.sensor[1], self.res, self.position, self.look, self.worldup)
        c2s = scale((1, 1, 1.0 / (self.far - self.near))) @ translate((0, 0, -self.near))   # Cameras.h:222-223
        return _camera_desc(capi.RT_CAMERA_ORTHOGRAPHIC, np.linalg.inv(c2s) @ r2s, c2w, r2s)


@dataclass
class PinholeCamera:
    """PinholeCamera(radius, box_dimensions, pos, look, right, worldup, res) (Cameras.h:313-359); the sampler
    overload of generateRay aims every ray at the hole's centre (0, 0, box_dimensions.z)."""
    radius: float = 1.0
    box: tuple = (36.0, 24.0, 50.0)
    position: tuple = (0.0, 0.0, 0.0)
    look: tuple = (0.0, 0.0, 1.0)
    right: tuple = (1.0, 0.0, 0.0)
    worldup: tuple = (0.0, 1.0, 0.0)
    res: tuple = (500, 500)

    def desc(self):
        r2s, c2w = _camera_base(self.box[0], self.box[1], self.res, self.position, self.look, self.worldup)
        return _camera_desc(capi.RT_CAMERA_PINHOLE, np.eye(4), c2w, r2s, pinhole_depth=float(self.box[2]))


@dataclass
class ThinlensCamera:
    """ThinlensCamera(R_curvature, lens_d, apeture, sensor_depth, sensor_w, sensor_h, pos, look, right, worldup,
    res) (Cameras.h:362-409): focal point F = R/2, aperture diameter lens_d - apeture."""
    curvature_radius: float = 100.0
    lens_diameter: float = 20.0
    aperture: float = 5.0
    sensor_depth: float = 60.0
    sensor: tuple = (36.0, 24.0)
    position: tuple = (0.0, 0.0, 0.0)
    look: tuple = (0.0, 0.0, 1.0)
    right: tuple = (1.0, 0.0, 0.0)
    worldup: tuple = (0.0, 1.0, 0.0)
    res: tuple = (500, 500)

    def desc(self):
        r2s, c2w = _camera_base(self.sensor[0], self.sensor[1], self.res, self.position, self.look, self.worldup)
        f32 = np.float32
        return _camera_desc(capi.RT_CAMERA_THINLENS, np.eye(4), c2w, r2s,
                            thin_focal=float(f32(self.curvature_radius) / f32(2.0)),
                            thin_aperture_diameter=float(f32(self.lens_diameter) - f32(self.aperture)),
                            sensor_depth=float(self.sensor_depth))


@dataclass
class PerspectiveCamera:
    """PerspectiveCamera(near, far, sensor_w, sensor_h, fov, pos, look, right, worldup, res, lens, focal)
    (Cameras.h:248-311).  `aspect_fix` (build-defined, default off = reference) builds the sensor as
    (w, w/aspect) instead of the reference's (w, w*aspect) (Cameras.h:255), for undistorted 16:9 frames."""
    near: float = 1.0
    far: float = 1000.0
    fov: float = 45.0
    position: tuple = (0.0, 0.0, 0.0)
    look: tuple = (0.0, 0.0, 1.0)
    right: tuple = (1.0, 0.0, 0.0)
    worldup: tuple = (0.0, 1.0, 0.0)
    res: tuple = (500, 500)
    lens_radius: float = 0.0
    focal_distance: float = 0.0
    aspect_fix: bool = False

    def matrices(self):
        N, F = self.near, self.far
        rx, ry = self.res
        t = math.tan(math.radians(self.fov) / 2.0)
        sw = 2 * N * t
        sh = sw * (rx / ry) if not self.aspect_fix else sw * (ry / rx)
        screen_to_ndc = scale((1 / sw, 1 / sh, 1)) @ translate((sw / 2, sh / 2, 0))   # Cameras.h:88-89
        ndc_to_raster = scale((rx, -ry, 1)) @ translate((0, -1, 0))                   # Cameras.h:90-91
        raster_to_screen = np.linalg.inv(ndc_to_raster @ screen_to_ndc)                # Cameras.h:93-94
        persp = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, F / (F - N), -(F * N / (F - N))], [0, 0, 1, 0]], float)
        inv_tan = 1.0 / t
        camera_to_screen = persp @ scale((inv_tan, inv_tan, 1))                        # Cameras.h:305-307
        raster_to_camera = np.linalg.inv(camera_to_screen) @ raster_to_screen          # Cameras.h:309
        d = np.asarray(self.look, float)
        d = d / np.linalg.norm(d)
        r = np.cross(np.asarray(self.worldup, float), d)
        r = r / np.linalg.norm(r)
        u = np.cross(d, r)                                                             # Cameras.h:130-139
        cam_to_world = np.eye(4)
        cam_to_world[:3, 0], cam_to_world[:3, 1], cam_to_world[:3, 2] = r, u, d
        cam_to_world[:3, 3] = self.position
        return raster_to_camera, cam_to_world

    def desc(self):
        r2c, c2w = self.matrices()
        return _camera_desc(capi.RT_CAMERA_PERSPECTIVE, r2c, c2w, lens_radius=self.lens_radius,
                            focal_distance=self.focal_distance)


# ------------------------------------------------------------------------------- sampler / film


@dataclass
class StratifiedSampler:
    """pbrt::StratifiedSampler(xPixelSamples, yPixelSamples, jitter, seed) (samplers.h:66-136)."""
    x_samples: int = 10
    y_samples: int = 10
    jitter: bool = False
    seed: int = 0

    def spp(self):
        return self.x_samples * self.y_samples

    def desc(self):
        return capi.rt_sampler_desc(capi.RT_SAMPLER_STRATIFIED, self.x_samples, self.y_samples, int(self.jitter), self.seed)


@dataclass
class SobolSampler:
    """pbrt::SobolSampler(samplesPerPixel, fullResolution, randomize, seed) (samplers.h:227-327); the film
    resolution comes from rt_film_set."""
    samples_per_pixel: int = 16
    randomize: int = capi.RT_SOBOL_FAST_OWEN
    seed: int = 0

    def spp(self):
        return self.samples_per_pixel

    def desc(self):
        return capi.rt_sampler_desc(capi.RT_SAMPLER_SOBOL, self.samples_per_pixel, 1, 0, self.seed, self.randomize)


@dataclass
class IndependentSampler:
    """pbrt::IndependentSampler(samplesPerPixel, seed) (samplers.h:38-62)."""
    samples_per_pixel: int = 16
    seed: int = 0

    def spp(self):
        return self.samples_per_pixel

    def desc(self):
        return capi.rt_sampler_desc(capi.RT_SAMPLER_INDEPENDENT, self.samples_per_pixel, 1, 0, self.seed)


# PixelSensor choices (rt_film_desc.sensor): "xyz" then the camera curves of spectrum.cpp, in the same order as
# tools/extract_spectra.py CAMERAS / rt_sensor_name
SENSORS = ["xyz", "canon_eos_100d", "canon_eos_1dx_mkii", "canon_eos_200d", "canon_eos_200d_mkii", "canon_eos_5d",
           "canon_eos_5d_mkii", "canon_eos_5d_mkiii", "canon_eos_5d_mkiv", "canon_eos_5ds", "canon_eos_m",
           "hasselblad_l1d_20c", "nikon_d810", "nikon_d850", "sony_ilce_6400", "sony_ilce_7m3", "sony_ilce_7rm3",
           "sony_ilce_9"]


@dataclass
class Film:
    """Film {film_dim, image_res, filter, pixel_sensor} (Film.h:11-20) with a BoxFilter/TriangleFilter of
    radius pixel_size/2 (RayTracerTestApp.h:143-147) and the XYZ PixelSensor's imagingRatio."""
    res: tuple = (500, 500)
    filter: int = capi.RT_FILTER_BOX
    filter_radius: tuple = (0.5, 0.5)
    imaging_ratio: float = float(np.float32(1.0) / np.float32(106.856895))
    filter_param: float = 0.0        # Gaussian sigma / Lanczos tau (0: the reference defaults 0.5 / 3)
    sensor: int = capi.RT_SENSOR_XYZ  # or 1..17: SENSORS (the reference's camera response curves)
    sensor_illum: int = capi.RT_ILLUM_D65

    def desc(self):
        d = capi.rt_film_desc()
        d.res_x, d.res_y = self.res
        d.filter = self.filter
        d.filter_radius[:] = list(self.filter_radius)
        d.imaging_ratio = self.imaging_ratio
        d.filter_param = self.filter_param
        d.sensor = self.sensor
        d.sensor_illum = self.sensor_illum
        return d

    def new_pixels(self):
        return np.zeros((self.res[0] * self.res[1], 4), dtype=np.float32)


@dataclass
class Integrator:
    kind: int = capi.RT_INTEGRATOR_REFERENCE
    max_depth: int = 5
    albedo_rgb: tuple = (0.5, 0.5, 0.5)

    def desc(self):
        d = capi.rt_integrator_desc()
        d.kind = self.kind
        d.max_depth = self.max_depth
        d.albedo_rgb[:] = list(self.albedo_rgb)
        return d


# ------------------------------------------------------------------------------- analytic shapes


@dataclass
class Shape:
    """Shape(name, rigidtransform) base (Shapes.h:172-207): ObjectToRender = rigid * permutation_y_z,
    RenderToObject = inverse (float64, rounded once), normal matrix = mat3(transpose(inverse(O2R)))."""
    rigid: np.ndarray
    material: int

    def _fill(self, d):
        o2r = np.asarray(self.rigid, float) @ PERM_YZ
        r2o = np.linalg.inv(o2r)
        d.object_to_render[:] = colmajor(o2r).tolist()
        d.render_to_object[:] = colmajor(r2o).tolist()
        d.normal_to_render[:] = np.asarray(r2o.T[:3, :3], float).T.astype(np.float32).reshape(-1).tolist()
        d.material = self.material


@dataclass
class Sphere(Shape):
    """Sphere(r, zmin=-r, zmax=r, phimax=360) (Shapes.h:209-432)."""
    radius: float = 1.0

    def desc(self, d):
        self._fill(d)
        d.type = capi.RT_SHAPE_SPHERE
        d.radius, d.zmin, d.zmax, d.phimax = self.radius, -self.radius, self.radius, 360.0


@dataclass
class Disk(Shape):
    """Disk(height, in_radius, out_radius, phimax=360) (Shapes.h:622-758); emits along object +z."""
    height: float = 0.0
    inner_radius: float = 0.0
    outer_radius: float = 1.0

    def desc(self, d):
        self._fill(d)
        d.type = capi.RT_SHAPE_DISK
        d.height, d.inner_radius, d.outer_radius, d.phimax = self.height, self.inner_radius, self.outer_radius, 360.0


@dataclass
class TriangleSimple(Shape):
    """TriangleSimple(p1, p2, p3) (Shapes.h:760-907), object space."""
    p: tuple = ((0, 0, 0), (1, 0, 0), (0, 1, 0))

    def desc(self, d):
        self._fill(d)
        d.type = capi.RT_SHAPE_TRIANGLE
        d.p[:] = [float(np.float32(x)) for v in self.p for x in v]


# ------------------------------------------------------------------------------------ meshes


@dataclass
class TriModel:
    """TriModel(name, rigidtransform, mesh, back_facing_cull, ...) (Shapes.h:1282-1320).  Holds the
    object-space mesh (one vertex per face corner, like assimp's flat GenNormals output) and the
    ObjectToRender = rigidtransform * permutation_y_z matrix."""
    positions: np.ndarray            # (nv, 3) float32
    normals: np.ndarray              # (nv, 3) float32
    indices: np.ndarray              # (nt, 3) uint32
    rigid: np.ndarray = field(default_factory=lambda: np.eye(4))
    cull_backfaces: bool = False
    cull_look: tuple = (0.0, 0.0, 1.0)
    octree_capacity: int = 40
    tri_material: np.ndarray = None
    materials: list = field(default_factory=list)   # (sigmoid c0,c1,c2, emission_scale[, type, eta])
    lights: list = field(default_factory=list)      # dict(type=QUAD: p, e1, e2, n, material | DISK: shape,
                                                    #      material | POINT: p, scale | DISTANT: dir, scale)
    shapes: list = field(default_factory=list)      # Sphere / Disk / TriangleSimple, after the octree

    def object_to_render(self):
        return np.asarray(self.rigid, float) @ PERM_YZ

    def desc(self):
        """Build the rt_scene_desc; the returned object keeps the numpy buffers alive."""
        o2r = self.object_to_render()
        n2r = np.linalg.inv(o2r).T[:3, :3]
        self._pos = np.ascontiguousarray(self.positions, dtype=np.float32)
        self._nrm = np.ascontiguousarray(self.normals, dtype=np.float32)
        self._idx = np.ascontiguousarray(self.indices, dtype=np.uint32)
        d = capi.rt_scene_desc()
        d.n_vertices = len(self._pos)
        d.positions = self._pos.ctypes.data_as(C.POINTER(C.c_float))
        d.normals = self._nrm.ctypes.data_as(C.POINTER(C.c_float))
        d.n_triangles = len(self._idx)
        d.indices = self._idx.ctypes.data_as(C.POINTER(C.c_uint32))
        d.object_to_render[:] = colmajor(o2r).tolist()
        d.normal_to_render[:] = np.asarray(n2r, float).T.astype(np.float32).reshape(-1).tolist()
        d.cull_backfaces = int(self.cull_backfaces)
        d.cull_look[:] = list(self.cull_look)
        d.octree_capacity = self.octree_capacity
        if self.tri_material is not None:
            self._mat = np.ascontiguousarray(self.tri_material, dtype=np.int32)
            d.tri_material = self._mat.ctypes.data_as(C.POINTER(C.c_int32))
        mats = self.materials or [((0.0, 0.0, 0.0), 0.0)]
        self._mats = (capi.rt_material * len(mats))()
        for i, m in enumerate(mats):
            c, e = m[0], m[1]
            self._mats[i].type = m[2] if len(m) > 2 else capi.RT_MAT_DIFFUSE
            self._mats[i].sigmoid[:] = [float(np.float32(x)) for x in c]
            self._mats[i].emission_scale = e
            self._mats[i].eta = m[3] if len(m) > 3 else 0.0
        d.n_materials = len(mats)
        d.materials = C.cast(self._mats, C.POINTER(capi.rt_material))
        if self.lights:
            self._lights = (capi.rt_light * len(self.lights))()
            for i, L in enumerate(self.lights):
                self._lights[i].type = L.get("type", capi.RT_LIGHT_QUAD)
                for k in ("p", "e1", "e2", "n", "dir"):
                    if k in L:
                        getattr(self._lights[i], k)[:] = [float(np.float32(x)) for x in L[k]]
                self._lights[i].scale = L.get("scale", 0.0)
                self._lights[i].shape = L.get("shape", -1)
                self._lights[i].material = L.get("material", -1)
            d.n_lights = len(self.lights)
            d.lights = C.cast(self._lights, C.POINTER(capi.rt_light))
        if self.shapes:
            self._shapes = (capi.rt_shape * len(self.shapes))()
            for i, s in enumerate(self.shapes):
                s.desc(self._shapes[i])
            d.n_shapes = len(self.shapes)
            d.shapes = C.cast(self._shapes, C.POINTER(capi.rt_shape))
        self._desc = d
        return d


def grey_sigmoid(g):
    """color.cpp:35-37 uniform branch: RGBSigmoidPolynomial(0, 0, (g - .5f) / sqrt(g (1 - g))) in float32."""
    g = np.float32(g)
    return (0.0, 0.0, float((g - np.float32(0.5)) / np.sqrt(g * (np.float32(1) - g))))


def _flat_mesh(faces_xyz):
    """(nt, 3, 3) float64 corner positions -> one-vertex-per-corner float32 mesh with flat normals."""
    p = np.asarray(faces_xyz, dtype=np.float64)
    n = np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0])
    n = n / np.linalg.norm(n, axis=1, keepdims=True)
    pos = p.astype(np.float32).reshape(-1, 3)
    nrm = np.repeat(n, 3, axis=0).astype(np.float32)
    idx = np.arange(len(pos), dtype=np.uint32).reshape(-1, 3)
    return pos, nrm, idx


def procedural_blob(frequency=32, radius=8.0, seed=1):
    """Seeded 'bunny-like' displaced geodesic icosphere: 20*frequency^2 triangles, watertight at the
    float level (shared points are computed once), outward winding, flat normals.  Stand-in for the
    reference's assimp-loaded meshes (RayTracerTestApp.h:70-73), which are not shipped."""
    rng = np.random.default_rng(seed)
    phi = (1 + 5 ** 0.5) / 2
    V = np.array([[-1, phi, 0], [1, phi, 0], [-1, -phi, 0], [1, -phi, 0], [0, -1, phi], [0, 1, phi],
                  [0, -1, -phi], [0, 1, -phi], [phi, 0, -1], [phi, 0, 1], [-phi, 0, -1], [-phi, 0, 1]], float)
    Fc = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
          (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
          (8, 6, 7), (9, 8, 1)]
    f = frequency
    K = 14
    waves = rng.normal(size=(K, 3)) * rng.uniform(1.0, 4.0, size=(K, 1))
    amps = rng.uniform(0.02, 0.08, size=K)
    phases = rng.uniform(0, 2 * np.pi, size=K)
    ears = [np.array([0.35, 0.25, 0.9]), np.array([-0.35, 0.25, 0.9])]
    cache = {}

    def point(a, b, c, i, j):
        w = {}
        for vid, wt in ((a, f - i - j), (b, i), (c, j)):
            if wt:
                w[vid] = w.get(vid, 0) + wt
        key = tuple(sorted(w.items()))
        if key not in cache:
            q = sum(V[vid] * (wt / f) for vid, wt in key)
            u = q / np.linalg.norm(q)
            r = 1.0 + float(np.sum(amps * np.sin(waves @ u + phases)))
            for e in ears:
                e = e / np.linalg.norm(e)
                r += 0.45 * math.exp(-((1 - float(u @ e)) / 0.02))
            cache[key] = u * (radius * r)
        return cache[key]

    tris = []
    for (a, b, c) in Fc:
        for i in range(f):
            for j in range(f - i):
                p00, p10, p01 = point(a, b, c, i, j), point(a, b, c, i + 1, j), point(a, b, c, i, j + 1)
                tris.append((p00, p10, p01))
                if i + j < f - 1:
                    p11 = point(a, b, c, i + 1, j + 1)
                    tris.append((p10, p11, p01))
    tris = np.array(tris)
    # orient outward
    cen = tris.mean(axis=1)
    nn = np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0])
    flip = np.einsum("ij,ij->i", nn, cen) < 0
    tris[flip] = tris[flip][:, [0, 2, 1]]
    return _flat_mesh(tris)


# ------------------------------------------------------------------- Cornell box (build-defined)
CORNELL_WHITE = grey_sigmoid(0.73)
# The Cornell box's red and green walls: sRGB (.63, .065, .05) and (.14, .45, .091) through RGBToSpectrumTable
# (color.cpp:26-72): the reference's trilinear lookup in the regenerated coefficient table (rt_rgb_to_sigmoid).
# Module attributes CORNELL_RED / CORNELL_GREEN, computed on first use (they need the built library and its table).
CORNELL_RGB = {"CORNELL_RED": (0.63, 0.065, 0.05), "CORNELL_GREEN": (0.14, 0.45, 0.091)}
_colour_cache = {}


def __getattr__(name):
    if name in CORNELL_RGB:
        if name not in _colour_cache:
            _colour_cache[name] = rgb_albedo(CORNELL_RGB[name])
        return _colour_cache[name]
    raise AttributeError(name)
CORNELL_LIGHT_SCALE = 25.0


def _quad(a, b, c, d):
    return [(a, b, c), (a, c, d)]


def _box(top, h):
    """Closed block from its 4 top corners (y = h) down to y = 0: top, 4 sides, bottom = 12 triangles."""
    t = [np.array(p, float) for p in top]
    b = [np.array([p[0], 0.0, p[2]]) for p in top]
    q = _quad(t[0], t[1], t[2], t[3])
    for k in range(4):
        q += _quad(b[k], t[k], t[(k + 1) % 4], b[(k + 1) % 4])
    q += _quad(b[3], b[2], b[1], b[0])
    return q


def cornell_box(blocks=True, extra=None):
    """Cornell box as triangles (standard 0..556 mm geometry): 5 walls (10 tris) + light quad (2) +
    short and tall block (12 + 12) = 36 triangles, one quad area light slightly below the ceiling.
    World space directly (rigid transform = permutation_y_z so that ObjectToRender = identity)."""
    W, R, G, L = 0, 1, 2, 3
    faces, mats = [], []

    def add(quads, m):
        for tri in quads:
            faces.append(tri)
            mats.append(m)
    P = lambda *v: np.array(v, float)
    add(_quad(P(552.8, 0, 0), P(0, 0, 0), P(0, 0, 559.2), P(549.6, 0, 559.2)), W)                 # floor
    add(_quad(P(556, 548.8, 0), P(556, 548.8, 559.2), P(0, 548.8, 559.2), P(0, 548.8, 0)), W)     # ceiling
    add(_quad(P(549.6, 0, 559.2), P(0, 0, 559.2), P(0, 548.8, 559.2), P(556, 548.8, 559.2)), W)   # back
    add(_quad(P(0, 0, 559.2), P(0, 0, 0), P(0, 548.8, 0), P(0, 548.8, 559.2)), G)                 # right (green)
    add(_quad(P(552.8, 0, 0), P(549.6, 0, 559.2), P(556, 548.8, 559.2), P(556, 548.8, 0)), R)     # left (red)
    ly = 548.7
    add(_quad(P(343, ly, 227), P(343, ly, 332), P(213, ly, 332), P(213, ly, 227)), L)             # light
    if blocks:
        add(_box([(130, 165, 65), (82, 165, 225), (240, 165, 272), (290, 165, 114)], 165), W)
        add(_box([(423, 330, 247), (265, 330, 296), (314, 330, 456), (472, 330, 406)], 330), W)
    n_fixed = len(faces)
    if extra is not None:  # (nt, 3, 3) world-space triangles, already outward-wound, white material
        for tri in extra:
            faces.append(tri)
            mats.append(W)
    faces = np.array(faces)
    # make every wall face the interior / light face downward: orient normals toward the box centre
    centre = np.array([278.0, 274.4, 279.6])
    cen = faces.mean(axis=1)
    nn = np.cross(faces[:, 1] - faces[:, 0], faces[:, 2] - faces[:, 0])
    is_wall = np.array([m != L for m in mats]) & (np.arange(len(faces)) < 10)
    flip = is_wall & (np.einsum("ij,ij->i", nn, centre - cen) < 0)
    lflip = (np.array(mats) == L) & (nn[:, 1] > 0)
    faces[flip | lflip] = faces[flip | lflip][:, [0, 2, 1]]
    # blocks: outward
    blk = (np.arange(len(faces)) >= 12) & (np.arange(len(faces)) < n_fixed)
    cmean = lambda f: f.reshape(-1, 3).mean(0) if len(f) else np.zeros(3)  # (no blocks: unused)
    bc = np.where(np.arange(len(faces))[:, None] < 24, cmean(faces[12:24]), cmean(faces[24:]))
    nn = np.cross(faces[:, 1] - faces[:, 0], faces[:, 2] - faces[:, 0])
    bflip = blk & (np.einsum("ij,ij->i", nn, cen - bc) < 0)
    faces[bflip] = faces[bflip][:, [0, 2, 1]]
    # object space = world with y/z swapped so that ObjectToRender = I * perm_yz maps it back
    obj = faces[:, :, [0, 2, 1]]
    pos, nrm, idx = _flat_mesh(obj)
    light = dict(p=(343.0, ly, 227.0), e1=(0.0, 0.0, 105.0), e2=(-130.0, 0.0, 0.0), n=(0.0, -1.0, 0.0), material=L)
    model = TriModel(pos, nrm, idx, rigid=np.eye(4), cull_backfaces=False, octree_capacity=40,
                     tri_material=np.array(mats, dtype=np.int32),
                     materials=[(CORNELL_WHITE, 0.0), (__getattr__("CORNELL_RED"), 0.0), (__getattr__("CORNELL_GREEN"), 0.0),
                                ((0.0, 0.0, 0.0), CORNELL_LIGHT_SCALE)],
                     lights=[light])
    return model


def cornell_camera(res):
    """Build-defined Cornell view through the reference PerspectiveCamera: eye (278, 273, -800), +z."""
    return PerspectiveCamera(near=1.0, far=5000.0, fov=62.0, position=(278.0, 273.0, -800.0), look=(0, 0, 1),
                             right=(1, 0, 0), worldup=(0, 1, 0), res=res, lens_radius=0.0, focal_distance=0.0,
                             aspect_fix=True)


# ----------------------------------------------------------------------------------- configs


def reference_model_matrix():
    """m1 = T(0,-40,800) * Ry(45) * Rx(-90) * S(15) (RayTracerTestApp.h:83-86)."""
    return translate((0, -40, 800)) @ rotate(45.0, (0, 1, 0)) @ rotate(-90.0, (1, 0, 0)) @ scale((15, 15, 15))


@dataclass
class Config:
    name: str
    model: TriModel
    camera: PerspectiveCamera
    sampler: object
    film: Film
    integrator: Integrator
    index_begin: int
    index_end: int

    def samples(self):
        return self.film.res[0] * self.film.res[1] * (self.index_end - self.index_begin)


def cfg0_reference(res=(500, 500), frequency=32, n_index=11):
    """the reference app's own workload (RayTracerTestApp.h:70-189) on a procedural
    ~20k-triangle mesh, BoxFilter (deterministic stand-in for the Triangle filter), indices 0..10."""
    pos, nrm, idx = procedural_blob(frequency=frequency, radius=8.0, seed=1)
    model = TriModel(pos, nrm, idx, rigid=reference_model_matrix(), cull_backfaces=True, cull_look=(0, 0, 1))
    cam = PerspectiveCamera(near=1.0, far=1000.0, fov=45.0, position=(0, 0, 0), look=(0, 0, 1), right=(1, 0, 0),
                            worldup=(0, 1, 0), res=res, lens_radius=50.0, focal_distance=800.0)
    return Config("cfg0_reference", model, cam, StratifiedSampler(10, 10, False, 0),
                  Film(res=res, filter=capi.RT_FILTER_BOX), Integrator(capi.RT_INTEGRATOR_REFERENCE), 0, n_index)


def cfg_cornell(res=(256, 256), spp_side=4, n_index=None, max_depth=5):
    """BASELINE configs[0]/[1]: Cornell box, stratified jittered spp_side^2 spp, diffuse + NEE."""
    cam = cornell_camera(res)
    n_index = spp_side * spp_side if n_index is None else n_index
    return Config(f"cornell_{res[0]}x{res[1]}_{spp_side * spp_side}spp", cornell_box(), cam,
                  StratifiedSampler(spp_side, spp_side, True, 0), Film(res=res, filter=capi.RT_FILTER_BOX),
                  Integrator(capi.RT_INTEGRATOR_PATH, max_depth=max_depth), 0, n_index)


def cfg3_blob(res=(1920, 1080), spp_side=16, n_index=None, max_depth=5, frequency=70):
    """BASELINE configs[2]: a seeded ~100k-triangle procedural 'bunny-like' mesh
    (20*70^2 = 98,000 triangles) standing on the floor of the Cornell box, lit by its quad area light;
    walls, light and mesh form ONE triangle model and one octree (TRIANGLE_CAPACITY 40)."""
    pos, _, idx = procedural_blob(frequency=frequency, radius=1.0, seed=1)
    tri = pos[idx].astype(np.float64)                      # unit-ish blob, object space
    lo = tri.reshape(-1, 3).min(0)
    s = 150.0
    world = tri * s + np.array([278.0, -lo[1] * s + 0.5, 280.0])
    model = cornell_box(blocks=False, extra=world)
    cam = cornell_camera(res)
    n_index = spp_side * spp_side if n_index is None else n_index
    return Config(f"cfg3_blob{len(idx)}_{res[0]}x{res[1]}_{spp_side * spp_side}spp", model, cam,
                  StratifiedSampler(spp_side, spp_side, True, 0), Film(res=res, filter=capi.RT_FILTER_BOX),
                  Integrator(capi.RT_INTEGRATOR_PATH, max_depth=max_depth), 0, n_index)


def mixed_scene(frequency=70):
    """SURVEY §8(d) CFG4 scene: the CFG3 procedural mesh (smaller, back right) in the Cornell box, three
    spheres — diffuse, perfect mirror, BK7 glass — and four lights: the ceiling quad, a disk under the ceiling,
    a point light and a sun shining in through the open front (build-defined placement constants)."""
    pos, _, idx = procedural_blob(frequency=frequency, radius=1.0, seed=1)
    tri = pos[idx].astype(np.float64)
    lo = tri.reshape(-1, 3).min(0)
    s = 105.0
    world = tri * s + np.array([370.0, -lo[1] * s + 0.5, 380.0])
    model = cornell_box(blocks=False, extra=world)
    W, R, G, L = 0, 1, 2, 3
    mats = list(model.materials)
    mats[L] = ((0.0, 0.0, 0.0), 12.0)                                            # ceiling quad: dimmer
    DIFF, MIRR, GLASS, DISKL = len(mats), len(mats) + 1, len(mats) + 2, len(mats) + 3
    mats += [(__getattr__("CORNELL_GREEN"), 0.0, capi.RT_MAT_DIFFUSE, 0.0),
             (grey_sigmoid(0.9), 0.0, capi.RT_MAT_MIRROR, 0.0),
             ((0.0, 0.0, 0.0), 0.0, capi.RT_MAT_DIELECTRIC, 0.0),                # eta 0 = glass-BK7
             ((0.0, 0.0, 0.0), 30.0)]
    model.materials = mats
    down = translate((150.0, 540.0, 430.0)) @ rotate(180.0, (1, 0, 0))             # disk normal -> -y
    model.shapes = [Sphere(translate((120.0, 60.0, 330.0)), DIFF, radius=60.0),
                    Sphere(translate((430.0, 70.0, 120.0)), MIRR, radius=70.0),
                    Sphere(translate((215.0, 65.0, 140.0)), GLASS, radius=65.0),
                    Disk(down, DISKL, height=0.0, inner_radius=0.0, outer_radius=40.0)]
    quad = dict(model.lights[0])
    quad["type"] = capi.RT_LIGHT_QUAD
    model.lights = [quad,
                    dict(type=capi.RT_LIGHT_DISK, shape=3),
                    dict(type=capi.RT_LIGHT_POINT, p=(450.0, 420.0, 250.0), scale=4.0e4),
                    dict(type=capi.RT_LIGHT_DISTANT, dir=(0.25, 0.6, -1.0), scale=1.5)]
    return model


def cfg4_mixed(res=(1920, 1080), spp=(32, 32), max_depth=5, frequency=70):
    """BASELINE configs[3]: mixed scene, NEE + MIS (power heuristic), 1024 spp."""
    cam = cornell_camera(res)
    return Config(f"cfg4_mixed_{res[0]}x{res[1]}_{spp[0] * spp[1]}spp", mixed_scene(frequency), cam,
                  StratifiedSampler(spp[0], spp[1], True, 0), Film(res=res, filter=capi.RT_FILTER_BOX),
                  Integrator(capi.RT_INTEGRATOR_PATH_MIS, max_depth=max_depth), 0, spp[0] * spp[1])


def cfg5_spectral(res=(3840, 2160), spp=(64, 32), max_depth=5, frequency=70):
    """BASELINE configs[4]: the CFG4 scene, 8 hero wavelengths per path, 4K, 2048 spp."""
    c = cfg4_mixed(res=res, spp=spp, max_depth=max_depth, frequency=frequency)
    c.name = f"cfg5_spectral_{res[0]}x{res[1]}_{spp[0] * spp[1]}spp"
    return c


# ------------------------------------------------------------------ ingest / colour / image output


def load_obj(path):
    """rt_load_obj: Wavefront OBJ -> (positions, normals, indices) as the reference's assimp import leaves a
    MeshCache::Mesh (AssetManager.cpp:67-190): triangulated, one vertex per corner, flat normals if absent."""
    lib = capi.load_library()
    m = C.POINTER(capi.rt_mesh)()
    rc = lib.rt_load_obj(str(path).encode(), C.byref(m))
    if rc != capi.RT_OK:
        raise capi.RTError("rt_load_obj", rc, f"cannot load {path}")
    try:
        mm = m.contents
        nv = mm.n_vertices
        pos = np.ctypeslib.as_array(mm.positions, shape=(nv, 3)).copy()
        nrm = np.ctypeslib.as_array(mm.normals, shape=(nv, 3)).copy()
        idx = np.ctypeslib.as_array(mm.indices, shape=(mm.n_triangles, 3)).copy()
    finally:
        lib.rt_mesh_free(m)
    return pos, nrm, idx


def rgb_albedo(rgb):
    """rt_rgb_to_sigmoid: RGBAlbedoSpectrum(sRGB, rgb) sigmoid coefficients — RGBToSpectrumTable::operator()
    (color.cpp:26-72) over the regenerated coefficient table."""
    lib = capi.load_library()
    src = (C.c_float * 3)(*[float(x) for x in rgb])
    out = (C.c_float * 3)()
    rc = lib.rt_rgb_to_sigmoid(src, out)
    if rc != capi.RT_OK:
        raise capi.RTError("rt_rgb_to_sigmoid", rc, f"rgb {rgb} outside [0,1]" if rc == capi.RT_E_ARG
                           else "coefficient table missing (python __graft_entry__.py build)")
    return tuple(float(x) for x in out)


def write_image(path, rgb8, res, flip_y=True):
    """rt_image_write: the resolved (res_x*res_y, 3) uint8 film to PNG / PPM, bottom row first by default."""
    lib = capi.load_library()
    a = np.ascontiguousarray(rgb8, np.uint8)
    rc = lib.rt_image_write(str(path).encode(), int(res[0]), int(res[1]), a.ctypes.data_as(C.POINTER(C.c_uint8)),
                            int(flip_y))
    if rc != capi.RT_OK:
        raise capi.RTError("rt_image_write", rc, f"cannot write {path}")
