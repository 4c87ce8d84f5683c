// Internal POD layouts shared by the host C-ABI layer (rt_host.cpp) and the HIP kernels (rt_kernels.hip).
//
// HBM layout (see DESIGN.md §Data layout):
//   octree nodes      : nodeA[n] = float4(pmin.xyz, bits(first_child | -1)), nodeB[n] = float4(pmax.xyz, 0)
//                       node order = the reference's creation order (Octtree_Model.h:351), children contiguous
//   leaf ranges       : int2 leafRange[set][n] = (first tile, count); set 0 = all triangles, set 1 = without
//                       back-facing triangles (TriModel::ComputeBackFace, Shapes.h:1339-1380)
//   triangle tiles    : 3 float4 per leaf reference, in leaf order: (p0.xyz,p1.x) (p1.yz,p2.xy) (p2.z,bits(id),0,0)
//                       world space (ObjectToRender applied once, Shapes.h:1117-1122), degenerate ones dropped
//   per triangle      : triWorld 3 float4, triNormal 3 float4 (object-space vertex normals), triMaterial int
//   sample streams    : SoA by sample s = i*n_pixels + j (i = index in batch, j = pixel slot in tile order)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace rtmi {

static const int kSpecN = 471;      // dense spectra 360..830 nm (spectrum.h:17, 380-381)
static const int kF1Max = 128;      // piecewise F1 entries (81 + 2 padding, spectrum.cpp:134-165)

struct DevSpectra {                 // Spectra::Init products (spectrum.cpp:2612-2634) + colour space illuminant
    float X[kSpecN], Y[kSpecN], Z[kSpecN], D65[kSpecN];
    float f1_lambda[kF1Max], f1_value[kF1Max];
    int f1_n;
    float bk7_lambda[kF1Max], bk7_value[kF1Max];   // glass-BK7 eta, FromInterleaved(.., false) (spectrum.cpp:2674)
    int bk7_n;
    float SR[kSpecN], SG[kSpecN], SB[kSpecN];      // the film's PixelSensor r_bar / g_bar / b_bar (dense)
    // the same dense values packed per wavelength, {SR, SG, SB, D65}[λ - 360]: the kernels stage it in LDS (7.5 KB)
    // and gather one ds_read_b128 per hero wavelength instead of a scattered global load per table (rt_kernels.hip)
    float4 SPK[kSpecN];
};

struct DevCamera {
    float r2c[16], c2w[16];         // column-major
    float lens_radius, focal_distance;
    int type;                       // RT_CAMERA_*
    float r2s[16];                  // M_RastertoScreen (pinhole / thin lens)
    float pinhole_depth, thin_focal, thin_aperture, sensor_depth;
};

struct DevSampler {
    int kind, xs, ys, jitter, seed, spp;
    // stratified with power-of-two xs and ys: the stratum split, PermutationElement's final modulo and the divisions
    // by xs / ys / spp become masks, shifts and multiplications by the exact reciprocals (same values)
    int p2, lg_xs;
    float inv_xs, inv_ys, inv_spp;
    int randomize, sobol_m, scale;  // SobolSampler (samplers.h:229-327)
    const uint32_t* sobol_mats;     // kSobolDims x kSobolMatrixSize generator columns
    const uint64_t* sobol_fwd;      // SobolIntervalToIndex tables for sobol_m (kSobolMatrixSize each)
    const uint64_t* sobol_inv;
};
static const int kSobolDims = 32, kSobolMatrixSize = 52;

// Division by an invariant divisor d for dividends 0 <= n < 2^31 (Granlund & Montgomery, Thm 4.2 with N = 31):
// l = ceil(log2 d), m = ceil(2^(31 + l) / d), n / d = (n m) >> (31 + l) exactly (n m < 2^63).  m == 0: unset.
struct IntDiv {
    uint64_t m = 0;
    int l = 0;
};
inline IntDiv make_intdiv(uint32_t d) {
    IntDiv r;
    if (d == 0) return r;
    int l = 0;
    while ((1ull << l) < d) ++l;
    r.l = l;
    r.m = ((1ull << (31 + l)) + d - 1) / d;
    return r;
}
__device__ __forceinline__ int intdiv(int n, const IntDiv& D) { return (int)(((uint64_t)(uint32_t)n * D.m) >> (31 + D.l)); }

struct DevFilm {
    int res_x, res_y, filter;
    IntDiv rx_div;  // pixel / res_x
    int y_int;      // 1: floorf((float)p / (float)res_x) == p / res_x for every pixel of the film (checked at film set)
    float rx, ry, imaging_ratio;
    const float* cdf_x;             // Gaussian / Lanczos: Continuous_Inversion_Sampler tables (N + 1 floats each)
    const float* cdf_y;
    int cdf_n;
};

struct DevLight {                   // rt_light (build-defined)
    float p[3], e1[3], e2[3], n[3];
    float area;
    int material;
    int type, shape;
    float dir[3];
    float scale;
    float ro, h;                    // disk: outer radius and height of shapes[shape]
    float o2r[16];                  // disk: ObjectToRender of shapes[shape]
};

struct DevMaterial {                // rt_material + the area light it feeds (MIS)
    float c0, c1, c2, emit;
    int type;
    float eta;
    int light;
    int cls;                        // material bin: 0 Lambert or emitter, 1 mirror or dielectric (kMatClasses)
};

struct DevShape {                   // rt_shape (Shapes.h:209-907)
    int type, material, light, pad;
    float r, zmin, zmax, h, ri, ro;
    float o2r[16], r2o[16], n2r[9];
    float p1[3], p2[3], p3[3];
    float bs[4];  // render-space bounding sphere of the shape: centre, padded radius^2 (rt_host.cpp shape_bound)
};

struct DevScene {
    const float4* nodeA;
    const float4* nodeB;
    const int2* leafRange[2];
    const float4* tiles[2];
    const float4* triWorld;
    const float4* triNormal;
    const int* triMaterial;
    const DevMaterial* materials;
    const DevShape* shapes;         // analytic shapes, intersected after the octree (prim id = n_tris + index)
    const DevLight* lights;
    int n_nodes;
    int n_tris;
    int n_shapes;
    int n_lights;
    int n_materials;                // entries of materials (>= 1)
    int mis;                        // RT_INTEGRATOR_PATH_MIS
    int full;                       // path shading needs the general kernel (shapes, specular, >1 / non-quad lights, MIS)
    DevLight light0;
    const float4* clusters[2];      // single-leaf scenes: (pmin, pmax) of each run of kClusterTris leaf tiles, inflated,
                                    // followed by the boxes of runs of kSuperClusters clusters
    int n_clusters[2];
    float4 cl_guard;                  // (centre, radius²): rays starting farther out never skip a cluster
    unsigned long long fan_pairs[2];  // single-leaf scenes: bit k (k even) = tiles k, k+1 are a fan pair (a,b,c),(a,c,d)
    int qcap;                       // BFS group FIFO size (compiled variants); 0 = global-memory ring below
    int depth;                      // octree depth (root = 0): any-hit queries walk depth-first when <= kDfsDepth
    // multi-level octrees: the rays the BVH leaves ambiguous are resolved in the kernel that found them by the
    // wave-cooperative BFS (rt_kernels.hip bfs_coop), whose FIFO holds kCoopFifo 16-bit group ids; coop_ok = the
    // octree's exact worst-case BFS queue (rt_octree_info max_queue_groups) fits it, so no fallback launch is needed
    int coop_ok;
    int* ring;                      // qcap == 0: ring[(pos & ring_mask) * ring_threads + thread]
    int ring_mask;
    int ring_threads;               // launches with qcap == 0 are clamped to this many threads
    // multi-level octrees (qcap != 1): the fast traversal's 8-wide compressed BVH per tile set (rt_bvh.cpp:
    // kBvhNodeF4 float4 per node) and its leaf-ordered triangle tiles (9 floats each, packed) with their triangle
    // ids; rays it finds ambiguous fall back to the octree BFS
    const float4* bvh[3];           // [0], [1]: closest-hit BVH of tile set 0 / 1; [kBvhAny]: the any-hit walks' BVH
    const float* btiles[3];         // ([kBvhAny]: its own build, SAH node cost 2; RTMI_BVH_ANY="0/4" aliases set 0's
    const int* btid[3];             // arrays, "cost/leaf" builds it with other parameters)
    float wabs;                     // canonical-rule window W(t) = t 2^-16 + wabs
    float oguard;                   // rays whose origin has a coordinate beyond +-oguard are ambiguous (the box
                                    // padding covers the slab test's rounding only for origins inside 8 M)
    unsigned amb_mask;              // test knob (RTMI_FORCE_AMB=k): with amb_force set, rays whose direction-bit hash
    int amb_force;                  // has its low k bits zero are declared ambiguous (exercises every fallback path)
    // the emissive surfaces (material emit > 0): non-degenerate triangle ids and shape indices, for the last depth's
    // emitter filter (k_emitter_filter); n_emit_tris < 0: too many emissive triangles, no filter
    const int* emit_tris;
    int n_emit_tris;
    const int* emit_shapes;
    int n_emit_shapes;
};
static const int kMaxEmitTris = 64;  // emitter filter only with at most this many emissive triangles
static const int kCoopFifo = 2048;   // entries of the wave-cooperative BFS's group FIFO (16-bit group ids, LDS)

// device counter slots (u64).  Every wave of a persistent kernel adds its totals at the end, all at about the same
// time: one counter word per slot serialised those atomics (a fixed ~0.15 ms tail per trace launch), so each slot
// is spread over kCtrSubs words, one per 256-B line, picked by wave; the host sums them (ctr_word, ctr_total).
#if RT_SIMD_STATS
void simd_stats_read(unsigned long long* out);  // rt_kernels.hip (measurement builds)
#endif
enum { C_NODES = 0, C_TRIS, C_HITS, C_RAYS, C_SHADOW, C_SAMPLES, C_SNODES, C_STRIS, C_FALLBACK, C_SFALLBACK,
       C_NEEVTX, C_COOPOVF, C_NCOUNTERS = 16 };  // C_COOPOVF: cooperative-BFS FIFO overflows (coop_ok: must stay 0)
constexpr int kCtrSubs = 32;   // words per counter slot
constexpr int kCtrLine = 32;   // u64 between words: 256 B
constexpr size_t kCtrWords = (size_t)C_NCOUNTERS * kCtrSubs * kCtrLine;
__host__ __device__ inline size_t ctr_word(int slot, int sub) { return ((size_t)slot * kCtrSubs + sub) * kCtrLine; }

// host: 8-wide compressed BVH build (rt_bvh.cpp; node layout there): kBvhNodeF4 float4 (128 B) per node.
// The top of every BVH is laid out breadth-first: nodes [0, kBvhTopNodes) (9 = the root and its children; 73 = three
// full levels), staged in LDS by the multi-level traversal kernels.
static const int kBvhNodeF4 = 8, kBvhNodeRead = 5;  // float4 per node / float4 the kernels read (N0..N4)
#ifndef RT_BVH_TOP_NODES
#define RT_BVH_TOP_NODES 9
#endif
static const int kBvhTopNodes = RT_BVH_TOP_NODES;
static_assert(kBvhTopNodes >= 9 && kBvhTopNodes <= 102, "staged top nodes: the root's children at least, 4 blocks per CU");
static const int kBvhMaxLeaf = 4;  // triangles per closest-hit leaf (SAH may stop earlier; r03 A/B with the speculative
                                   // walk: 4 vs 8 CFG3 +1 %, CFG4 +1.1 %; 5, 6 between)
static const int kBvhAny = 2;                         // DevScene bvh / btiles index of the any-hit BVH
struct BvhData {
    std::vector<float4> nodes;
    std::vector<float> tiles;  // 9 floats per tile (p0, p1, p2), leaf order
    std::vector<int> tid;      // triangle id per tile
    int depth = 0, max_leaf = 0;
};
void build_bvh8(const float* tri9, const int* ids, int n, float pad, float node_cost, BvhData& out,
                int max_leaf = kBvhMaxLeaf);
// compact tiles (9 floats + id) -> the exported 12-float view (p0.xyz, p1.x) (p1.yz, p2.xy) (p2.z, bits(id), 0, 0)
void bvh_tiles_logical(const float* t9, const int* tid, int n, float* out12);

}  // namespace rtmi

// ---------------------------------------------------------------------------------------------------
// Kernel I/O descriptors and host launch wrappers (defined in rt_kernels.hip)

namespace rtmi {

struct SampleIds {
    const int* work_pixels;  // owned pixel ids in tile order
    int n_pixels;            // pixels per sample index
    int index_begin;
    const int* ex_pixel;     // explicit (pixel, index) pairs (parity entry point) or nullptr
    const int* ex_index;
    IntDiv np_div;           // s / n_pixels (unset: plain division)
};

// Path state of a slot (path mode): 8 float4 fields — λ[8] at R_LAM.., β[8] at R_BETA.., L[8] at R_L.., the PCG
// state (uint2) and, in the record layout, the pixel id at R_RNG (the increment is recomputed from the pixel hash),
// (dimension, prevPdf, TerminateSecondary flag, pixel id) at R_MISC — at p + f * fs + slot * ss.  Multi-level
// scenes, whose coherence sort leaves slots scattered over a wave, store a slot as ONE 128-B record (fs 1, ss 8):
// one cache line per access instead of one per field (CFG3 +10 %, CFG4 +8 %).  Single-leaf scenes keep their
// slots almost in queue order and store the fields SoA (fs n, ss 1): a wave's field access stays coalesced (the
// record layout cost the Cornell box 7 %).  The pdfs stay SoA (pdfA/pdfB): only TerminateSecondary and the film
// read them.
enum { R_LAM = 0, R_BETA = 2, R_L = 4, R_RNG = 6, R_MISC = 7, kRecF4 = 8 };
struct RecView {
    float4* p;
    size_t fs;    // float4s between fields
    unsigned ss;  // float4s between slots
    int rng8;     // 1: the R_RNG field holds only the 8-byte PCG state per slot, densely (uint2 array; SoA simple path
                  // scenes), the increment is recomputed from the pixel hash; 0: state + increment (uint4)
};

struct GenOut {
    float4* rayO; float4* rayD;   // the origin's w = the ray's path slot
    float4* lamA; float4* lamB; float4* pdfA; float4* pdfB;  // reference mode (lamA/lamB) + pdfs
    RecView rec;                                             // path mode: the slot state (λ, sampler, β, L, ...)
    int lean;  // no β = 1 / L = 0 / pdf stores (depth 0 and the film kernel derive them); 1: the simple path, which
               // stores no dimension either (the host derives each depth's); 2: mixed scenes (dimension, prevPdf = 0
               // and the TerminateSecondary flag 0 in R_MISC)
    int rsh = 0;  // ray k at rayO[k << rsh] / rayD[k << rsh] (1: the workspace's interleaved (o, d) pairs)
    // path mode: the batch's two queue-counter regions (2 kQRegion ints), zeroed by this kernel instead of a memset
    // launch (in two-lane mode every launch of a lane may wait for the other lane's resident blocks)
    int* zero = nullptr;
};

// Ray queues are split into kShards shards, each with its own length and chunk-ticket counters: one returning
// device-scope atomic word saturates at ~88 operations/us (MI355X_MICROARCH "dequeue"), and a 16 Mi-ray bounce makes
// 65 k block appends (single leaf) or 262 k wave tickets + appends (multi-level) per launch.  Shard j of a queue
// holds positions [j S, j S + len_j); a kernel processes the items of shard j into shard j of its output queue, so
// an output shard never outgrows S.  Blocks prefer shard blockIdx % kShards (blocks are dealt round-robin to the 8
// XCDs), waves drain other shards when theirs is empty.
static const int kShards = 8;
// Queue counters: one 256-B line each (never two hot atomics in one cache line), in a region of kQRegion ints:
// per shard the queue length, the chunk tickets of its trace and shade launches, and the shadow-queue length and
// chunk ticket (multi-level octrees).  Counter x of shard j is at x + j * kQStride.
static const int kQStride = 64;
enum { kQLen = 0, kQTraceTicket = 1 * kShards * kQStride, kQShadeTicket = 2 * kShards * kQStride,
       kQShadowLen = 3 * kShards * kQStride, kQShadowTicket = 4 * kShards * kQStride,
       kQNeeFallback = 5 * kShards * kQStride,
       // material bins of a mixed multi-level scene's bounce (TraceIO bin_*): class c's shard lengths at
       // kQBinLen + c kShards kQStride, the chunk tickets of its shade kernel at kQBinTicket + c kShards kQStride
       kQBinLen = 6 * kShards * kQStride, kQBinTicket = 8 * kShards * kQStride,
       kQTraceFallback = 10 * kShards * kQStride,  // the trace kernel's ambiguous-ray list length (TraceIO fb_len)
       kQRegion = 11 * kShards * kQStride };
static const int kMatClasses = 2;  // material bins: 0 Lambert or emitter (NEE), 1 mirror or dielectric
// Shard stride of a queue of ns shards for n items (a multiple of 64, so wave chunks stay line-aligned); capacity
// ns * S.  Single-leaf scenes (static chunks, one block append per 256 rays) keep one shard: sharding their queues
// cost the Cornell box 3 %; multi-level scenes (per-wave tickets and appends) use kShards (CFG3 +5.5 %).
inline __host__ __device__ int shard_stride(int n, int ns) {
    int s = (n + ns - 1) / ns;
    return (s + 63) & ~63;
}
// A queue of ns shards: shard lengths at len[j * kQStride], or len == nullptr for the dense queue of n items in
// positions [0, n) (shard j = [j S, min(n, (j + 1) S))).
struct QueueView {
    const int* len;
    int S;
    int n;
    int ns;
};
static const int kBlockThreads = 256;  // threads per block of every kernel
static const int kClusterTris = 2;     // leaf tiles per culling cluster (single-leaf scenes; 4 or 6: -2 %)

struct TraceIO {
    const float4* rayO; const float4* rayD;
    QueueView q;              // the queue's shards
    int set;                  // tile set: 0 = all triangles, 1 = back-face culled
    float4* hitB;             // (b0, b1, b2, t) at the ray's queue position
    int* hitPrim;
    int* ticket = nullptr;    // per-shard chunk tickets (zeroed before the launch) or nullptr: static chunks
    int rsh = 0;              // ray k at rayO[k << rsh] (1: the workspace's interleaved (o, d) pairs; 0: caller arrays)
    // sorted bounce (multi-level scenes, tickets only): position p traces the queue's ray perm[p] (rt_sort.hip) and
    // stores it to so[2p], so[2p + 1] — the sorted side queue the shade kernel reads; nullptr: no sort
    const int* perm = nullptr;
    float4* so = nullptr;
    // multi-level scenes in path mode: the trace kernel walks the BVH alone and lists the queue positions of the rays
    // the canonical rule cannot decide here; k_trace_fallback then runs the exact BFS for them (so the
    // trace kernel holds no BFS registers).  nullptr: the BFS runs inline (reference mode, debug entry points).
    int* fb_pos = nullptr;
    int* fb_len = nullptr;
    // path mode, depths >= 1: the next queue's counter region (kQRegion ints), zeroed by block 0 of this kernel
    // instead of a memset launch (no kernel of the depth touches it before the shade that appends to it)
    int* zero = nullptr;
};

// Material binning of a mixed multi-level scene's bounce (k_bin_materials, after the trace): every hit's queue
// position is appended to the index list of its material class (idx[c], sharded like the queue, shard lengths at
// len + c kShards kQStride); misses are appended to no bin (no miss work in the full path integrator).
struct BinIO {
    QueueView q;             // the traced queue
    const int* hitPrim;
    int* idx[kMatClasses];
    int* len;
    // lean depth 0 (GenOut lean): k_generate left L unwritten, so the misses' L = 0 is stored here (no bin sees them);
    // rayO == nullptr otherwise.  Queue rays are interleaved (o, d) pairs: ray k's origin (w = slot) at rayO[2k].
    const float4* rayO = nullptr;
    RecView rec{};
};
hipError_t launch_bin_materials(hipStream_t st, int grid, const DevScene& sc, const BinIO& io);

// The last depth of a mixed scene (depth == max_depth > 0): only hits on an emitter still add to L, so the rays that
// hit no emissive surface at all — each emitter tested alone with tMax = FLT_MAX, a test the closest-hit traversal's
// own test of that surface can only pass if this one does (both are monotone in tMax) — are dropped before the trace
// (k_emitter_filter).  The others are appended, shard by shard, to the output queue (interleaved (o, d) pairs).
struct EmitIO {
    QueueView q;              // the depth's queue
    const float4* rayO;       // its rays: ray k at rayO[2k], rayO[2k + 1]
    float4* nO;               // the filtered queue (same shard stride), lengths at nCount + j kQStride (zeroed)
    int* nCount;
};
hipError_t launch_emitter_filter(hipStream_t st, int grid, const DevScene& sc, const EmitIO& io);

struct ShadeRefIO {
    const int* work_pixels; int n_pixels; int n_index;
    const float4* rayD; const float4* lamA; const float4* lamB; const float4* pdfA; const float4* pdfB;
    const float4* hitB; const int* hitPrim;
    float4* film;
    float albedo_c2, illum_c2, illum_scale;
    int rsh;  // ray k at rayD[k << rsh]
};

// Coherence-sort key parameters of the bounce rays a shade kernel appends (ray_sort_key below).
struct RayKeyIO {
    unsigned* key = nullptr;  // per next-queue position; nullptr: no sort
    float4 lo, scale;         // origin quantisation: (p - lo) * scale in [0, 512)
    int dir_bits = 0, org_bits = 0, org_major = 0;
};
struct PathIO {
    // queue rays are interleaved (o, d) pairs, 32 B per ray: ray k at rayO[2k] / rayD[2k] (rayD = rayO + 1), nO / nD too
    const float4* rayO; const float4* rayD; QueueView q;  // current queue (origin w = the ray's path slot)
    const float4* hitB; const int* hitPrim;                                     // at queue position
    float4* nO; float4* nD; int* nCount;  // next queue: same shard stride, lengths at nCount + j kQStride
    RecView rec;                                                          // slot state (R_LAM ...)
    float4* pdfA; float4* pdfB;                                           // TerminateSecondary writes them
    int depth, max_depth;
    int lean;   // k_generate ran lean (GenOut::lean): depth 0 starts from β = 1, L = 0 in registers; 2: the pdfs are
                // not stored either, TerminateSecondary sets R_MISC's z instead (k_path_film recomputes the pdfs)
    int dim;    // >= 0: the sampler dimension every path of this depth starts from (simple path: each bounce takes
                // two Get2D); -1: per slot in R_MISC
    int* ticket;  // per-shard chunk tickets (zeroed before the launch) or nullptr: static chunks
    RayKeyIO nkey;  // multi-level scenes: the coherence-sort key of every appended ray (rt_sort.hip)
    const int* bin_idx = nullptr;  // material-binned shade: item i of q is queue position bin_idx[i] (BinIO)
};

// Shadow queue (multi-level octrees): the shade kernel appends NEE shadow rays {o, tMax}, {d, slot} and their
// pending contribution instead of tracing them inline; k_path_shadow traces them.  shO == nullptr: inline.  Sharded
// like the ray queues (same stride; lengths and tickets at shCount / shTicket + j kQStride).
// A separate trailing kernel argument, so PathIO (and the single-leaf kernels' code) is unchanged.
struct ShadowQueueIO {
    float4 *shO = nullptr, *shD = nullptr, *shLA = nullptr, *shLB = nullptr;
    int *shCount = nullptr, *shTicket = nullptr;
    // 1: the shade kernel traces its NEE shadow rays inline over the BVH and queues only the ambiguous ones (the
    // canonical rule could not decide: §6b) for k_path_shadow, which runs the exact traversal; 0: every shadow ray
    // is queued (RTMI_SHADOW_QUEUE=1).  Multi-level simple-path scenes always have a queue.
    int defer = 0;
};

// Deferred NEE of the mixed-scene shade: k_path_shade_full samples every light at a Lambert vertex (same sampler
// dimensions and order as inline) and leaves one NEE record per slot — {po.xyz, bits(material | bounced << 31)}, the
// lights' sample points (u0, u1) two per float4, then the light weights four per float4 (< 0: the light is skipped,
// cos <= 0) — and appends the slot to the NEE queue (sharded like the ray queues, counters at kQShadowLen /
// kQShadowTicket).  k_path_nee re-derives each light's shadow ray (wi, tMax) from (po, u0, u1) with the same code,
// traces a vertex's shadow rays in light order and adds the visible lights' terms to L in that order, so L is
// bit-identical to the inline loop.  It also owns the vertex's throughput update: the shade kernel leaves β as it
// was, k_path_nee forms x = β (R / π) for the light terms (R = the material's reflectance at λ) and, when the cosine
// bounce continued the path (`bounced`), stores β R.  A 4-light record is 64 B (round 3: 128 B of rays and x[8]).
// The traversals do not share a kernel with the path state (CFG4: 198 VGPRs unbudgeted, 464-656 B/lane spill under
// the 4-wave budget).
inline __host__ __device__ int nee_stride(int n_lights) { return 1 + (n_lights + 1) / 2 + (n_lights + 3) / 4; }  // float4s
enum { N_PO = 0, N_UV = 1 };  // the weights at N_UV + ceil(n / 2)
struct NeeIO {
    float4* rec;   // NEE records, nee_stride(n_lights) float4s per slot; nullptr: inline NEE (not used)
    int* slot;     // NEE queue: slot per position (same shard stride as the ray queues)
    int* len;      // shard lengths (zeroed with the queue's counter region)
    int* ticket;   // per-shard chunk tickets of k_path_nee
    int* fb_slot;  // multi-level scenes: slots of the vertices whose shadow rays the BVH alone could not decide,
    int* fb_len;   // re-run by k_path_nee<Q, true> with the exact traversal (their count: zeroed with the region)
    unsigned* key; // NEE sort (nullptr: none): the Morton code of the shading point per NEE queue position
    float4 lo, scale; int key_bits;  // its quantisation (SortRaysIO lo / scale) and bits per axis
};

// 9 bits -> every third bit of 27
__device__ __forceinline__ unsigned spread3_9(unsigned v) {
    v &= 0x1ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
// Morton code of p quantised as (p - lo) * scale in [0, 512), `bits` per axis (the coherence sorts' origin keys)
__device__ __forceinline__ unsigned morton_key(float x, float y, float z, float4 lo, float4 scale, int bits) {
    auto q = [](float v) {
        v = v < 0.f ? 0.f : (v > 511.f ? 511.f : v);
        return (unsigned)v;
    };
    return spread3_9(q((x - lo.x) * scale.x) >> (9 - bits)) << 2 | spread3_9(q((y - lo.y) * scale.y) >> (9 - bits)) << 1 |
           spread3_9(q((z - lo.z) * scale.z) >> (9 - bits));
}

// Coherence-sort key of a bounce ray (rt_sort.hip; DESIGN.md §6 key table): direction octant, the direction's cell
// on a 2^dir_bits x 2^dir_bits octahedral grid, and the origin's Morton code with org_bits per axis — origin-major
// (org_major) or direction-major.  Written by the shade kernels beside every appended ray.
__device__ __forceinline__ unsigned ray_sort_key(float4 p, float4 v, const RayKeyIO& k) {
    const unsigned oct = (v.x < 0.f ? 4u : 0u) | (v.y < 0.f ? 2u : 0u) | (v.z < 0.f ? 1u : 0u);
    const float sum = fabsf(v.x) + fabsf(v.y) + fabsf(v.z);
    const float G = (float)(1 << k.dir_bits);
    const unsigned ux = (unsigned)fminf(fabsf(v.x) / sum * G, G - 1), uy = (unsigned)fminf(fabsf(v.y) / sum * G, G - 1);
    const unsigned mo = morton_key(p.x, p.y, p.z, k.lo, k.scale, k.org_bits);
    const unsigned dk = oct << (2 * k.dir_bits) | ux << k.dir_bits | uy;
    return k.org_major ? (mo << (3 + 2 * k.dir_bits)) | dk : (dk << (3 * k.org_bits)) | mo;
}

struct PathFilmIO {
    const int* work_pixels; int n_pixels; int n_index;
    RecView rec; const float4* pdfA; const float4* pdfB;
    float4* film;
    int lean;  // pdf = VisibleWavelengthsPDF(λ) recomputed here; 2: and divided as TerminateSecondary did when the
               // slot's R_MISC z flag is set (mixed scenes: dispersive glass)
};

struct RecordIO {
    int n;
    const float4* rayO; const float4* rayD; const float4* lamA; const float4* lamB; const float4* pdfA;
    const float4* pdfB; const float4* hitB; const int* hitPrim;
    float* out; int stride;  // rt_sample_record (floats)
    int rsh = 0;             // ray k at rayO[k << rsh]
};

hipError_t launch_generate(hipStream_t st, int grid, int nS, const SampleIds& ids, const DevCamera& cam,
                           const DevSampler& smp, const DevFilm& film, const GenOut& out);
hipError_t launch_trace_closest(hipStream_t st, int grid, int qcap, const DevScene& sc, const TraceIO& io,
                                unsigned long long* ctr);
// the rays k_trace_closest listed in io.fb_pos (multi-level scenes; a small grid, the list's length read on the device)
hipError_t launch_trace_fallback(hipStream_t st, int grid, int qcap, const DevScene& sc, const TraceIO& io,
                                 unsigned long long* ctr);
hipError_t launch_occluded(hipStream_t st, int qcap, const DevScene& sc, int n, const float4* o, const float4* d,
                           int* out, unsigned long long* ctr, bool path = false);
// Coherence sorts (rt_sort.hip): stable device radix sorts with no host read.  temp = sort_temp_bytes() bytes.
struct SortRaysIO {
    const unsigned* qkey;                                 // ray keys at the queue positions (ray_sort_key, written
                                                          // by the shade kernel that appended the rays)
    int* perm;                                            // out: sorted position -> queue position (the trace
                                                          // kernel gathers the rays: TraceIO perm)
    unsigned* keys; unsigned* keys_alt; int* vals; int* vals_alt;
    void* temp;
    int dir_bits, org_bits;                               // key: octant, 2 x dir_bits direction, 3 x org_bits origin
    int* len;     // the queue's shard lengths (kQLen region): read, then rewritten for the sorted queue
    int S;        // shard stride (the sorted queue keeps it; its shards split the sorted order evenly)
};
size_t sort_temp_bytes();
hipError_t launch_sort_rays(hipStream_t st, const SortRaysIO& io);
struct SortNeeIO {
    int* slot; int* len; int S;                          // the NEE queue (NeeIO slot / len), sorted in place
    const unsigned* key;                                 // per queue position, written by k_path_shade_full (NeeIO key)
    unsigned* keys; unsigned* keys_alt; int* vals; int* vals_alt;
    void* temp;
    int org_bits;                                        // key: 3 x org_bits Morton code of the shading point
};
hipError_t launch_sort_nee(hipStream_t st, const SortNeeIO& io);
hipError_t launch_oct_classify(hipStream_t st, int nnodes, const float* cbox, const int* seg, const int* ent,
                               const float* tri9, unsigned char* mask, int* stats);
hipError_t launch_oct_scatter(hipStream_t st, int njobs, int nchild, const int* job, const int* ent,
                              const unsigned char* mask, int* ent_next, int* s0);
hipError_t launch_ref_shade_film(hipStream_t st, int grid, const DevScene& sc, const DevSpectra* sp, const DevFilm& film,
                                 const ShadeRefIO& io, unsigned long long* ctr);
hipError_t launch_records(hipStream_t st, const DevScene& sc, const DevSpectra* sp, const DevFilm& film,
                          const ShadeRefIO& sio, const RecordIO& io);
hipError_t launch_path_shadow(hipStream_t st, int grid, int qcap, bool dfs, const DevScene& sc, const PathIO& io,
                              const ShadowQueueIO& shq, unsigned long long* ctr);
// matclass (mixed scenes): 0 every material in one kernel; 1 / 2 the Lambert-or-emitter / specular bin (io.bin_idx)
hipError_t launch_path_shade(hipStream_t st, int grid, int qcap, const DevScene& sc, const DevSpectra* sp,
                             const DevSampler& smp, const DevFilm& film, const SampleIds& ids, const PathIO& io,
                             unsigned long long* ctr, const ShadowQueueIO& shq = ShadowQueueIO{},
                             const NeeIO& nee = NeeIO{}, int matclass = 0);
hipError_t launch_path_film(hipStream_t st, int grid, const DevSpectra* sp, const DevFilm& film, const PathFilmIO& io,
                            unsigned long long* ctr);
hipError_t launch_path_nee_fallback(hipStream_t st, int grid, int qcap, const DevScene& sc, const DevSpectra* sp,
                                    const PathIO& io, const NeeIO& nee, unsigned long long* ctr);
hipError_t launch_path_nee(hipStream_t st, int grid, int qcap, const DevScene& sc, const DevSpectra* sp,
                           const PathIO& io, const NeeIO& nee, unsigned long long* ctr);
hipError_t launch_resolve(hipStream_t st, int n, const float4* film, const float* m_xyz_from_sensor,
                          const float* m_rgb_from_xyz, unsigned char* out, int srgb);
hipError_t launch_film_gather(hipStream_t st, int n, const int* work, const float4* film, float4* out);
hipError_t launch_film_scatter(hipStream_t st, int n, const int* work, const float4* in, float4* film);

}  // namespace rtmi
