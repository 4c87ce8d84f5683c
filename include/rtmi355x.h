/* =====================================================================================================
 * rtmi355x.h — the drop-in C-ABI of the MI355X ray-tracing inner loop (librtmi355x.so).
 *
 * Replaces the in-process per-pass block of the reference application
 *     RayTracerTestApp::MainLoop  →  ThreadFunction / evaluate_pixel dispatch + wait
 *     (Applications/RayTracerTestApp.h:287-422)
 * which samples (sampler), generates camera rays (CameraBase::generateRay, Cameras.h:179/273-297),
 * traverses the triangle octree (Octtree_Model::Traverse, Octtree_Model.h:66-127), shades (Li lambda,
 * RayTracerTestApp.h:218-284) and accumulates sensor RGB into the Film (Film.h:11-20, :336-337).
 *
 * Plain C: pointers and sizes only.  All descriptors are deep-copied at upload; the caller owns every
 * buffer.  Every entry point returns 0 (RT_OK) or a negative rt_status and sets rt_last_error().
 * No C++ exception crosses this boundary.  One rt_ctx per host thread (calls on a context are
 * serialised by the caller).  The library needs an MI355X (gfx950): rt_create fails with
 * RT_E_NODEVICE when none is present — there is no CPU fallback.
 * ===================================================================================================*/
#ifndef RTMI355X_H
#define RTMI355X_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 9

typedef enum {
    RT_OK = 0,
    RT_E_ARG = -1,      /* invalid argument / descriptor                                   */
    RT_E_HIP = -2,      /* HIP runtime error (message in rt_last_error)                    */
    RT_E_RCCL = -3,     /* reserved: collectives run in the caller (torch.distributed)     */
    RT_E_OOM = -4,      /* device or host allocation failed (std::bad_alloc is caught)     */
    RT_E_STATE = -5,    /* call order: scene/camera/sampler/film not set; internal error   */
    RT_E_NODEVICE = -6, /* no gfx950 device visible                                        */
    RT_E_LIMIT = -7     /* scene exceeds a compiled limit (e.g. BFS queue bound)           */
} rt_status;

typedef struct rt_ctx rt_ctx;

#define RT_MAX_DEVICES 16
#define RT_QUEUE_SHARDS 8   /* shards of the multi-level path queues (rt_debug_sort) */
/* rt_create ("device list"): n_devices <= 1 renders on `device`; n_devices > 1 renders every pass
 * on devices[0..n_devices) at once — pixel tiles interleaved over the devices (tile t -> device t mod n), the
 * caller's film on devices[0] (rt_render_pass_device) or on the host, owned pixels exchanged with peer copies
 * over xGMI.  The film is bit-identical to a one-device render.  A device may be listed more than once (tests). */
typedef struct {
    int device;        /* HIP device ordinal (n_devices <= 1)                             */
    int octree_build;  /* RT_OCTREE_BUILD_DEVICE (default) or RT_OCTREE_BUILD_HOST         */
    int n_devices;     /* 0 or 1: one device; 2..RT_MAX_DEVICES: devices[]                 */
    int devices[RT_MAX_DEVICES];
    int reserved[5];
} rt_options;
/* Where rt_scene_upload builds the octree (Octtree_Model.h:33-63): both give the reference's tree bit for bit. */
enum { RT_OCTREE_BUILD_DEVICE = 0, RT_OCTREE_BUILD_HOST = 1 };

/* Film pixel, layout-identical to `pixel {glm::vec3 rgbsum; float weightsum;}` (Film.h:6-9). */
typedef struct { float r, g, b, w; } rt_pixel;

enum { RT_MAT_DIFFUSE = 0, RT_MAT_MIRROR = 1, RT_MAT_DIELECTRIC = 2 };
/* Build-defined material (the reference has none: Shading.h:1-21 is a comment stub).
 * DIFFUSE: Lambert R/π; MIRROR: perfect specular reflection scaled by R; R(λ) is an RGBSigmoidPolynomial
 *   (color.h:363-403): R(λ) = s(c0 λ² + c1 λ + c2).
 * DIELECTRIC: smooth Fresnel glass; eta > 0 is a constant IOR, eta == 0 selects the dispersive
 *   "glass-BK7" table (spectrum.cpp:2674-2691) with SampledWavelengths::TerminateSecondary (spectrum.h:302-310).
 * emission_scale > 0 makes the surface a pure one-sided emitter with Le = scale · stdillum-D65. */
typedef struct {
    int type;
    float sigmoid[3];
    float emission_scale;
    float eta;
} rt_material;

enum { RT_SHAPE_SPHERE = 0, RT_SHAPE_DISK = 1, RT_SHAPE_TRIANGLE = 2 };
/* Analytic shapes besides the triangle octree (Shapes.h:172-907), intersected in object space.
 * SPHERE: Sphere(r, zmin, zmax, phimax) (Shapes.h:209-432) — full spheres only (zmin <= -r, zmax >= r,
 *   phimax >= 360), so the atan2 φ clip can never fire;  DISK: Disk(height, inner, outer, phimax)
 *   (Shapes.h:622-758), phimax >= 360;  TRIANGLE: TriangleSimple(p1, p2, p3) (Shapes.h:760-907). */
typedef struct {
    int type;
    float object_to_render[16];      /* column-major rigidtransform * permutation_y_z (Shapes.h:175-181) */
    float render_to_object[16];      /* column-major glm::inverse(ObjectToRender)                        */
    float normal_to_render[9];       /* column-major mat3(transpose(inverse(ObjectToRender))) (:150)     */
    float radius, zmin, zmax, phimax;
    float height, inner_radius, outer_radius;
    float p[9];                      /* TriangleSimple p1, p2, p3 (object space) */
    int material;
} rt_shape;

enum { RT_LIGHT_QUAD = 0, RT_LIGHT_DISK = 1, RT_LIGHT_POINT = 2, RT_LIGHT_DISTANT = 3 };
/* Build-defined lights (Lights.h:1-10 is a comment stub naming area, point and sun lights).
 * QUAD: x = p + u·e1 + v·e2, emitting normal n, Le from `material` (the quad is also geometry: two
 *   emissive triangles of the mesh);  DISK: uniform area sampling of shapes[shape] (an emissive DISK
 *   shape with inner_radius 0), Le from its material;  POINT: at p, intensity scale · D65;
 *   DISTANT: unit direction `dir` towards the light, irradiance scale · D65. */
typedef struct {
    int type;
    float p[3], e1[3], e2[3], n[3];
    float dir[3];
    float scale;
    int shape;
    int material;
} rt_light;

/* TriModel + Octtree_Model inputs (Shapes.h:1272-1491, Octtree_Model.h:33-63). */
typedef struct {
    int n_vertices;
    const float* positions;          /* object space, 3 floats per vertex (MeshCache::Mesh::positions) */
    const float* normals;            /* object space vertex normals (MeshCache::Mesh::normals)        */
    int n_triangles;
    const uint32_t* indices;         /* 3 per triangle                                                 */
    float object_to_render[16];      /* column-major; = rigidtransform * permutation_y_z (Shapes.h:180) */
    float normal_to_render[9];       /* column-major mat3(transpose(inverse(ObjectToRender))) (:1364)   */
    int cull_backfaces;              /* TriModel::ComputeBackFace(look, enable) (Shapes.h:1339-1380)    */
    float cull_look[3];
    int octree_capacity;             /* TRIANGLE_CAPACITY (Octtree_Model.h:388); 0 -> 40                */
    const int32_t* tri_material;     /* per triangle material id, NULL -> 0 (path integrator only)     */
    int n_materials;
    const rt_material* materials;
    int n_lights;
    const rt_light* lights;
    int n_shapes;                    /* analytic shapes, intersected after the octree in list order     */
    const rt_shape* shapes;
} rt_scene_desc;

enum { RT_CAMERA_PERSPECTIVE = 0, RT_CAMERA_ORTHOGRAPHIC = 1, RT_CAMERA_PINHOLE = 2, RT_CAMERA_THINLENS = 3 };
/* The values CameraBase and its subclasses already hold (Cameras.h:190-210 and the members below).
 * PERSPECTIVE: generateRay Cameras.h:273-297 (raster_to_camera, lens_radius, focal_distance);
 * ORTHOGRAPHIC: Cameras.h:230-243 (raster_to_camera);
 * PINHOLE: Cameras.h:328-339, the sampler overload (raster_to_screen, pinhole_depth = box_dimensions.z);
 * THINLENS: Cameras.h:378-400 (raster_to_screen, thin_focal = R/2, thin_aperture_diameter = lens_d - apeture,
 *   sensor_depth); the reference only offers a (lens_angle, len_percent_r) overload, so the build draws one
 *   Get2D per sample: lens_angle = 360° · u0, len_percent_r = u1. */
typedef struct {
    int type;
    float raster_to_camera[16];      /* column-major M_RastertoCamera */
    float camera_to_world[16];       /* column-major M_CameratoWorld  */
    float lens_radius;
    float focal_distance;
    float raster_to_screen[16];      /* column-major M_RastertoScreen (Cameras.h:93-94) */
    float pinhole_depth;
    float thin_focal;
    float thin_aperture_diameter;
    float sensor_depth;
} rt_camera_desc;

enum { RT_SAMPLER_INDEPENDENT = 0, RT_SAMPLER_STRATIFIED = 1, RT_SAMPLER_SOBOL = 2 };
enum { RT_SOBOL_NONE = 0, RT_SOBOL_PERMUTE_DIGITS = 1, RT_SOBOL_FAST_OWEN = 2, RT_SOBOL_OWEN = 3 };
/* pbrt::IndependentSampler(spp, seed) (samplers.h:38-62): x_samples = spp, y_samples ignored.
 * pbrt::StratifiedSampler(x, y, jitter, seed) (samplers.h:66-136).
 * pbrt::SobolSampler(spp, film resolution, randomize, seed) (samplers.h:227-327): x_samples = spp.  The
 * reference declares SobolMatrices32 without defining it (HelperFunctions.h:208-210); the build generates the
 * generator matrices for 32 dimensions from the Joe-Kuo direction numbers (dimensions >= 32 wrap to 2 as in
 * samplers.h:270-283) and derives SobolIntervalToIndex's VdC tables itself (equal to HelperFunctions.h:212-470). */
typedef struct {
    int kind;
    int x_samples, y_samples;
    int jitter;
    int seed;
    int randomize;                   /* Sobol: RT_SOBOL_* */
} rt_sampler_desc;

enum { RT_FILTER_BOX = 0, RT_FILTER_TRIANGLE = 1, RT_FILTER_GAUSSIAN = 2, RT_FILTER_LANCZOS = 3 };
/* PixelSensor (pixelsensor.h:37-79).  RT_SENSOR_XYZ: r/g/b = CIE X/Y/Z, XYZFromSensorRGB = WhiteBalance(sensor
 * illuminant white -> sRGB white).  1..17: the camera response curves the reference names in spectrum.cpp
 * (rt_sensor_name), XYZFromSensorRGB fitted over the 24 Macbeth swatches under the sensor illuminant exactly as
 * pixelsensor.h:37-68 does it (glm column-major LinearLeastSquares, helpers.h:258-272). */
enum { RT_SENSOR_XYZ = 0, RT_SENSOR_CANON_EOS_100D = 1, RT_SENSOR_COUNT = 18 };
/* Named illuminants of Spectra::Init (spectrum.cpp:2620-2637, all Y-normalised): the sensor illuminant. */
enum {
    RT_ILLUM_D65 = 0, RT_ILLUM_A = 1, RT_ILLUM_D50 = 2, RT_ILLUM_F1 = 3, /* F1..F12 = 3..14 */
    RT_ILLUM_ACES_D60 = 15, RT_ILLUM_COUNT = 16
};
/* Film (Film.h:11-20) + its filter + XYZ PixelSensor (pixelsensor.h:70-87).  Filters: Box (filters.h:66-93),
 * Triangle (267-296, deterministic coin), Gaussian (96-154, sigma = filter_param) and LanczosSinc (223-264,
 * tau = filter_param), the last two sampled through the reference's tabulated Continuous_Inversion_Sampler
 * (Sampling.h:781-877; 10000 / 2000 bins) driven by the sampler's GetPixel2D. */
typedef struct {
    int res_x, res_y;
    int filter;
    float filter_radius[2];
    float imaging_ratio;             /* 1/CIE_Y_integral in the reference app (RayTracerTestApp.h:149) */
    float filter_param;              /* Gaussian sigma (0 -> 0.5) / Lanczos tau (0 -> 3)               */
    int sensor;                      /* RT_SENSOR_XYZ or a camera (1..RT_SENSOR_COUNT-1)               */
    int sensor_illum;                /* RT_ILLUM_*: sensorIllum of the PixelSensor constructors        */
} rt_film_desc;

enum { RT_INTEGRATOR_REFERENCE = 0, RT_INTEGRATOR_PATH = 1, RT_INTEGRATOR_PATH_MIS = 2 };
/* RT_INTEGRATOR_REFERENCE: the Li lambda of RayTracerTestApp.h:218-284 (ambient 0.3·F1 +
 *   clamp(n·(0,0,-1))·D65·albedo), octree back-face culling honoured.
 * RT_INTEGRATOR_PATH: build-defined path tracer (Integrator.h:1-14 is a stub): one light
 *   sample per light at every diffuse vertex (NEE), emitters seen by camera rays or specular bounces.
 * RT_INTEGRATOR_PATH_MIS: the same plus BSDF-sampled emitter hits, both weighted by the power heuristic. */
typedef struct {
    int kind;
    int max_depth;
    float albedo_rgb[3];             /* reference Li material colour (grey: color.cpp:35-37 branch) */
} rt_integrator_desc;

typedef struct {
    int64_t samples;                 /* camera samples evaluated                         */
    int64_t rays;                    /* closest-hit rays traced                          */
    int64_t shadow_rays;             /* any-hit rays traced                              */
    int64_t nodes_tested;            /* box tests executed by closest-hit rays (BVH child boxes, plus octree
                                        nodes of BFS-traced rays)                        */
    int64_t tris_tested;             /* triangle tests executed by closest-hit rays      */
    int64_t shadow_nodes_tested;     /* node box tests by any-hit (shadow) rays          */
    int64_t shadow_tris_tested;      /* triangle tests by any-hit (shadow) rays          */
    int64_t hits;                    /* closest-hit rays that hit                        */
    double ms_generate, ms_trace, ms_shade, ms_shadow, ms_film;  /* HIP-event kernel time (0 with
                                        RTMI_NO_STAGE_EVENTS); ms_shadow is the deferred NEE kernel of mixed
                                        scenes or the shadow-queue kernel (RTMI_SHADOW_QUEUE=1), else 0: the
                                        simple path traces its shadow rays inside the shade kernel */
    int64_t launches_trace;          /* closest-hit trace launches (per-launch averages) */
    int64_t launches_shade;          /* shade launches (path mode: includes the inline shadow rays) */
    int64_t fallback_rays;           /* multi-level octrees: closest-hit rays the fast BVH traversal found
                                        ambiguous (canonical rule), traced by the reference BFS */
    int64_t shadow_fallback_rays;    /* the same for any-hit (shadow) rays                */
    double ms_sort;                  /* multi-level octrees: coherence sort of bounce rays (HIP events)  */
    int64_t nee_vertices;            /* mixed scenes: path vertices whose light samples k_path_nee traced */
    int64_t coop_overflows;          /* multi-level octrees: rays whose wave-cooperative BFS ran out of FIFO while the
                                        octree's exact queue bound promised it could not (DevScene coop_ok); always 0
                                        unless that bound is wrong — the tests require 0 */
} rt_stats;   /* multi-device contexts: every field summed over the devices */

/* Per-sample record for parity (stage outputs of one (pixel, index) camera sample). */
typedef struct {
    float lambda[8], pdf[8];
    float ro[3], rd[3];
    int32_t prim;
    float b[3], t;
    float L[8];
    float rgb[3];
    float weight;
} rt_sample_record;

/* Flattened octree as uploaded (node order = reference creation order, Octtree_Model.h:351). */
typedef struct {
    int n_nodes;
    int n_leaf_refs;
    int max_queue_groups;            /* host-computed bound of the BFS group queue       */
    int depth;
    int bvh_nodes;                   /* multi-level octrees: 4-wide nodes of the fast traversal's BVH (0: none) */
    int bvh_depth;
} rt_octree_info;

/* ---- lifecycle ---------------------------------------------------------------------------------- */
int rt_create(const rt_options* opt, rt_ctx** out);
void rt_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);
int rt_abi_version(void);

/* ---- configuration (each deep-copies its descriptor) -------------------------------------------- */
int rt_scene_upload(rt_ctx* ctx, const rt_scene_desc* scene);
int rt_camera_set(rt_ctx* ctx, const rt_camera_desc* cam);
int rt_sampler_set(rt_ctx* ctx, const rt_sampler_desc* smp);
int rt_film_set(rt_ctx* ctx, const rt_film_desc* film);
int rt_integrator_set(rt_ctx* ctx, const rt_integrator_desc* integ);
/* Pixel-tile sharding for multi-GPU: this context renders tiles t with t % n_shards == shard_id
 * (tile_size x tile_size pixel tiles in row-major tile order).  Default: one shard. */
int rt_set_shard(rt_ctx* ctx, int tile_size, int n_shards, int shard_id);

/* ---- the hot path ----------------------------------------------------------------------------- */
/* Accumulate (+=) sample indices [index_begin, index_end) of every owned pixel into film_inout
 * (res_x*res_y rt_pixel, host memory), index-ordered per pixel exactly as the reference's passes
 * (RayTracerTestApp.h:336-337, 420-422).  Blocks until done. */
int rt_render_pass(rt_ctx* ctx, int index_begin, int index_end, rt_pixel* film_inout);
/* Same, into a device-resident film (res_x*res_y rt_pixel in HBM) on the given hipStream_t
 * (NULL = the context's stream).  Returns after enqueueing; the caller synchronises. */
int rt_render_pass_device(rt_ctx* ctx, int index_begin, int index_end, void* d_film, void* hip_stream);

/* a20 resolve (RayTracerTestApp.h:424-452): rgbsum/weightsum -> XYZFromSensorRGB -> sRGB -> clamp -> u8. */
int rt_film_resolve(rt_ctx* ctx, const rt_pixel* film, uint8_t* rgb_out);

/* a20 + pbrt ColorEncoding::sRGB (color.h:537-557, commented out in the reference): the same resolve, quantised with
 * LinearToSRGB8 (enoki minimax polynomial, round-to-nearest) instead of the reference's linear 255·x truncation. */
int rt_film_resolve_srgb(rt_ctx* ctx, const rt_pixel* film, uint8_t* rgb_out);

/* ---- scene ingest / image output / colour (host only: no device needed) ------------------------------- */
/* MeshCache::Mesh as the reference's assimp import leaves it (AssetManager.cpp:67-190): triangulated, one
 * vertex per face corner, file normals or flat face normals (aiProcess_GenNormals), texcoords or 0. */
typedef struct {
    int n_vertices;
    float* positions;                /* 3 per vertex */
    float* normals;                  /* 3 per vertex */
    float* texcoords;                /* 2 per vertex */
    int n_triangles;
    uint32_t* indices;               /* 3 per triangle */
} rt_mesh;
/* Wavefront OBJ (v / vt / vn / f, polygons fan-triangulated, negative indices) -> *out (free with rt_mesh_free). */
int rt_load_obj(const char* path, rt_mesh** out);
void rt_mesh_free(rt_mesh* mesh);
/* Write w x h 8-bit RGB to `path`: PNG when it ends in .png, binary PPM otherwise; flip_y writes rows bottom-up
 * (the film's row 0 is the image bottom: the reference uploads it as a GL texture, RayTracerTestApp.h:453-455). */
int rt_image_write(const char* path, int w, int h, const uint8_t* rgb, int flip_y);
/* RGBToSpectrumTable::operator() (color.cpp:26-72) for an sRGB reflectance in [0,1]^3: grey = the closed form of
 * color.cpp:35-37, otherwise the reference's trilinear lookup in the 3 x 64^3 coefficient table, which the build
 * regenerates (the reference's "../rgb2spec/sRGB64binary", color.cpp:114, is not in its repository; data/srgb64.rgbspec,
 * found next to the library or through RTMI_RGBSPEC_TABLE).  RT_E_STATE when the table is missing. */
int rt_rgb_to_sigmoid(const float* rgb, float* coeffs);
/* The table generator's per-entry solve for one colour: Gauss-Newton in CIELAB (rgb2spec_opt's method). */
int rt_rgb_fit_sigmoid(const float* rgb, float* coeffs);
/* Name of a PixelSensor (RT_SENSOR_XYZ -> "xyz", 1.. -> the reference's camera name), NULL when out of range. */
const char* rt_sensor_name(int sensor);
/* The film's resolve matrices (column-major, glm layout): XYZFromSensorRGB of the current sensor, sRGB RGBFromXYZ. */
int rt_film_matrices(rt_ctx* ctx, float* xyz_from_sensor9, float* rgb_from_xyz9);

/* ---- instrumentation ---------------------------------------------------------------------------- */
int rt_get_stats(rt_ctx* ctx, rt_stats* out);
int rt_reset_stats(rt_ctx* ctx);
int rt_octree_get_info(rt_ctx* ctx, rt_octree_info* out);
/* Copy out the flattened octree: node_bounds[6*n] (pmin,pmax), node_child[n] (first child or -1),
 * node_leaf_first[n], node_leaf_count[n], leaf_refs[n_leaf_refs] (triangle ids incl. culled ones). */
int rt_octree_export(rt_ctx* ctx, float* node_bounds, int32_t* node_child, int32_t* node_leaf_first,
                     int32_t* node_leaf_count, int32_t* leaf_refs);
/* The fast multi-level traversal's 8-wide compressed BVH as uploaded: set 0 / 1 the closest-hit BVH of tile set 0 (all
 * triangles) / 1 (without back faces), set 2 the any-hit BVH of the shadow rays (all triangles), DESIGN.md §6b: *n_nodes nodes of 32 floats (128 B, layout in rt_bvh.cpp), *n_tiles triangle tiles of
 * 12 floats, consts[2] = (wabs, oguard) of the canonical rule.  Counts always; arrays when non-NULL.  Not a
 * reference structure (the reference traverses only its octree): exported so tests can replay the GPU's walk. */
int rt_bvh_export(rt_ctx* ctx, int set, int* n_nodes, int* n_tiles, float* consts, float* nodes, float* tiles);
/* The same BVH built on the host from a scene descriptor, without a context or a device (CPU tests). */
int rt_debug_bvh_build(const rt_scene_desc* scene, int set, int* n_nodes, int* n_tiles, float* consts, float* nodes,
                       float* tiles);

/* ---- parity entry points (same kernels as the hot path, stage outputs exposed) ------------------ */
/* K2 alone: closest hit of n world-space rays (ro, rd: 3n floats).  prim[n] (-1 = miss),
 * bt[4n] = (b0, b1, b2, t).  use_cull follows the reference's back-face flags. */
int rt_debug_trace(rt_ctx* ctx, int n, const float* ro, const float* rd, int use_cull, int32_t* prim, float* bt);
/* The path integrator's shadow query alone: any hit of n rays within (0, tmax[i]) against the octree and the
 * analytic shapes (Octtree_Model.h:66-127 with the early exit, Shapes.h shape tests); occluded[n] = 0 / 1. */
int rt_debug_occluded(rt_ctx* ctx, int n, const float* ro, const float* rd, const float* tmax, int32_t* occluded);
/* K1..K3 for n explicit (pixel_id, index) samples (reference integrator). */
int rt_debug_samples(rt_ctx* ctx, int n, const int32_t* pixel_ids, const int32_t* indices, rt_sample_record* out);
/* The multi-level coherence sorts alone (rt_sort.hip: stable device LSD radix sorts) on a synthetic queue of
 * RT_QUEUE_SHARDS shards of stride S (a multiple of 64): shard j holds shard_len[j] <= S items at positions
 * [j S, j S + shard_len[j]), with keys[pos] (8 S entries) and, for the NEE sort, slots[pos].  which 0: the bounce-ray
 * sort (key bits 3 + 2 bits_a + 3 bits_b; out[pos'] = the queue position of the sorted item at pos'); which 1: the
 * NEE-vertex sort (key bits 3 bits_a; out = the slots, sorted in place).  Sorted item k' sits at position
 * (k' / S2) S + k' % S2, S2 = ceil(ceil(n / 8) / 64) 64; out_len[8] = the rewritten shard lengths.  Not a
 * reference function (the reference has no sort): exported so tests can check order and stability directly. */
int rt_debug_sort(rt_ctx* ctx, int which, int S, const int32_t* shard_len, const uint32_t* keys, const int32_t* slots,
                  int bits_a, int bits_b, int32_t* out, int32_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* RTMI355X_H */
