// HIP kernels of the MI355X wavefront ray tracer (gfx950, wave64) + their host launch wrappers.
//
// Stage map:
//   k_generate        a1-a8   sampler → wavelengths → filter → thin-lens camera ray (SoA ray / λ / pdf streams)
//   k_trace_closest   a9-a12  Octtree_Model::Traverse: exact BFS order, shrinking tMax, watertight test
//   k_ref_shade_film  a13,a16-a19 reference Li + ToSensorRGB + clamp + Film accumulate (pixel-owned, index order)
//   k_path_shade      a22     build-defined diffuse path step: emission, NEE with the shadow ray traced inline
//                             (any-hit traversal, fixed tMax), cosine BSDF sample appended to the next queue
//   k_path_film       a18-a19 sensor + film for path mode
//   k_resolve         a20     film → sRGB u8
// Kernels are persistent-style grid-stride loops over wavefront queues whose lengths live in device memory
// (no host round trip between bounces); ray compaction is wave64 ballot + LDS prefix + one atomic per block
// and dominant-axis bin, so trace waves see one watertight-test permutation.
#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "rt_device.h"

namespace rtmi {

static constexpr int kBlock = kBlockThreads;
// Tuning constants (A/B measurements of the alternatives: DESIGN.md §4 levers table)
static constexpr int kLeafChunk = 32;  // triangles per leaf phase of the while-while traversal (16: -5 %, 64: +-0)
static constexpr int kLdsQ = 32;       // LDS-resident BFS group FIFO entries per lane (2 B each: 16 KB per block)
static constexpr int kTriUnroll = 4;   // triangles per scalar-cache batch in single-leaf traversal
#ifndef RT_BVH_STACK
#define RT_BVH_STACK 16
#endif
static constexpr int kBvhStack = RT_BVH_STACK;  // BVH traversal stack entries per lane (child word, entry distance): 32 KB
// One per block, shared by every multi-level traversal call site: the BVH stacks, and — for the rare rays the BVH
// hands to the reference BFS, after the wave's BVH loop has finished — that BFS's LDS-resident group FIFO.
__shared__ uint2 g_bstk[kBvhStack * kBlock];
static_assert(sizeof(uint2) * kBvhStack >= 2 * kLdsQ, "the BFS FIFO lives in the BVH stack's LDS");
// The any-hit walks' stacks: child words only (nothing to cull with a fixed tMax), 24 per lane: 24 KB per block, so
// the any-hit kernels (shade, NEE) are not held to 4 blocks per CU by LDS.  The BFS FIFO stays in g_bstk.
#ifndef RT_ANY_STACK
#define RT_ANY_STACK 24
#endif
static constexpr int kAnyStack = RT_ANY_STACK;
__shared__ unsigned g_astk[kAnyStack * kBlock];

// Single-leaf scenes, closest-hit waves without a shared dominant axis (bounce rays): pass 1 runs on a compacted list
// of (ray, cluster) pairs whose box test passes (wave ballot + prefix into LDS) instead of every cluster for every lane.
static constexpr int kCompactMaxClusters = 24;  // clusters of a compacted single leaf (Cornell: 18)
struct CompactWave {
    float4 ra[64], rb[64];                     // staged TriRay per lane: (Sx, Sy, Sz, ox), (oy, oz, kz, -)
    unsigned long long cand[64];               // pass-1 candidate mask per lane (leaf order bit k = tile k)
    unsigned short pair[64 * kCompactMaxClusters];  // lane | cluster << 6
};
__shared__ CompactWave g_cmp[kBlock / 64];  // one per wave, shared by every single-leaf traversal call site
// the single leaf's tiles (<= 64 triangles, 3 KB) and its culling clusters' boxes (<= 32, 1 KB) staged in LDS at
// kernel start by every kernel that traverses it
__shared__ float4 g_leaf1[3 * 64];
__shared__ float4 g_cl1[2 * 32];
__device__ __forceinline__ void stage_leaf1(const DevScene& sc, int set) {
    const int2 r = sc.leafRange[set][0];
    if (r.y <= 64)
        for (int i = threadIdx.x; i < 3 * r.y; i += blockDim.x) g_leaf1[i] = sc.tiles[set][3 * r.x + i];
    if (sc.n_clusters[set] <= 32)
        for (int i = threadIdx.x; i < 2 * sc.n_clusters[set]; i += blockDim.x) g_cl1[i] = sc.clusters[set][i];
    __syncthreads();
}
#define RT_LEAF1(tiles, base, j) (g_leaf1 + 3 * (j))
// multi-level scenes: the BVH's breadth-first top levels (kBvhTopNodes 8-wide nodes, the 80 B the kernels read of
// each; rt_bvh.cpp emit_root), which every ray opens, staged in LDS at kernel start by every kernel that traverses
// the BVH
__shared__ float4 g_top[kBvhNodeRead * kBvhTopNodes];
// ANY: the kernel's BVH walks are any-hit queries, which walk the any-hit BVH (sc.bvh[kBvhAny]); otherwise the
// closest-hit BVH of tile set `set`
__device__ __forceinline__ void simd_init();  // (RT_SIMD_STATS measurement builds, below)
template <int QCAP, bool ANY = true>
__device__ __forceinline__ void stage_scene(const DevScene& sc, int set) {
    if constexpr (QCAP == 1) {
        stage_leaf1(sc, set);
    } else {
        // (the host pads every node array to at least kBvhTopNodes nodes)
        const float4* b = sc.bvh[ANY ? kBvhAny : set];
        if (b)
            for (int i = threadIdx.x; i < kBvhNodeRead * kBvhTopNodes; i += blockDim.x)
                g_top[i] = b[(i / kBvhNodeRead) * kBvhNodeF4 + i % kBvhNodeRead];
        simd_init();
        __syncthreads();
    }
}
// An 8-wide node as the kernels read it (rt_bvh.cpp): header N0, N1 and the quantised child planes per axis.
struct BvhNode8 {
    float4 N0;
    uint4 N1, QX, QY, QZ;
};
__device__ __forceinline__ uint4 as_u4(float4 v) {
    return make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w));
}
__device__ __forceinline__ BvhNode8 load_node8(const float4* __restrict__ nodes, int node) {
    // one generic pointer (LDS top levels or global): five flat 16-B loads.  Two explicit paths (ds_read /
    // global_load) compiled to six global loads per node, the phi of the two paths splitting the last quantised
    // plane (r05_ab15: CFG3 +2.2 %, CFG4 +1.2 % with the flat loads)
    const float4* N = node < kBvhTopNodes ? g_top + kBvhNodeRead * node : nodes + (size_t)kBvhNodeF4 * node;
    return BvhNode8{N[0], as_u4(N[1]), as_u4(N[2]), as_u4(N[3]), as_u4(N[4])};
}
// the simple path's per-triangle shading inputs on single-leaf scenes (<= 64 triangles): world vertices and the
// material's (c0, c1, c2, emission), staged in LDS by k_path_shade<1>
__shared__ float4 g_tri1[4 * 64];
__device__ __forceinline__ bool stage_tris1(const DevScene& sc) {
    const bool ok = sc.n_tris <= 64;
    if (ok)
        for (int i = threadIdx.x; i < sc.n_tris; i += blockDim.x) {
            g_tri1[4 * i] = sc.triWorld[3 * i];
            g_tri1[4 * i + 1] = sc.triWorld[3 * i + 1];
            g_tri1[4 * i + 2] = sc.triWorld[3 * i + 2];
            const DevMaterial dm = sc.materials[sc.triMaterial[i]];
            g_tri1[4 * i + 3] = make_float4(dm.c0, dm.c1, dm.c2, dm.emit);
        }
    __syncthreads();
    return ok;
}
// Mixed-scene material table in LDS (<= kLdsMats entries, 32 B each): the shade and binning kernels look up the
// material of every hit (prim -> triMaterial -> material), so staging the table removes the chain's last global
// round trip.  Larger tables stay in global memory (mat_at reads through the pointer).
static constexpr int kLdsMats = 64;
__shared__ DevMaterial g_mat[kLdsMats];
__device__ __forceinline__ bool stage_materials(const DevScene& sc) {
    const bool ok = sc.n_materials <= kLdsMats;
    if (ok)
        for (int i = threadIdx.x; i < sc.n_materials; i += blockDim.x) g_mat[i] = sc.materials[i];
    __syncthreads();
    return ok;
}
__device__ __forceinline__ DevMaterial mat_at(const DevScene& sc, bool lds, int m) {
    if (lds) return g_mat[m];
    return sc.materials[m];
}
__device__ __forceinline__ int mbcnt64(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// -------------------------------------------------------------------------------- wave helpers
__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// SIMD efficiency of the BVH walks (measurement builds only, -DRT_SIMD_STATS=1): per slot pair, the lanes a wave
// step could have used (64 per step) and the lanes active in it; slots 0/1 closest-hit node tests, 2/3 closest-hit
// triangle tests, 4/5 any-hit node tests, 6/7 any-hit triangle tests.  Block sums in LDS, flushed by the trace and
// shade kernels; the host prints them with the stats (rt_host.cpp get_stats_one).
#ifndef RT_SIMD_STATS
#define RT_SIMD_STATS 0
#endif
#if RT_SIMD_STATS
__shared__ unsigned long long g_simd[8];
__device__ unsigned long long g_simd_glob[8];
__device__ __forceinline__ void simd_tick(int slot) {
    const uint64_t m = __ballot(1);
    if (lane_id() == __builtin_ctzll(m)) {
        atomicAdd(&g_simd[slot], 64ull);
        atomicAdd(&g_simd[slot + 1], (unsigned long long)__popcll(m));
    }
}
__device__ __forceinline__ void simd_init() {
    if (threadIdx.x < 8) g_simd[threadIdx.x] = 0;
}
__device__ __forceinline__ void simd_flush() {
    __syncthreads();
    if (threadIdx.x < 8) atomicAdd(&g_simd_glob[threadIdx.x], g_simd[threadIdx.x]);
}
void simd_stats_read(unsigned long long* out) {
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_simd_glob), sizeof(g_simd_glob));
}
#define RT_SIMD_TICK(s) simd_tick(s)
#else
#define RT_SIMD_TICK(s)
__device__ __forceinline__ void simd_init() {}
__device__ __forceinline__ void simd_flush() {}
#endif

// Append the `pred` lanes of a wave to a queue: one atomicAdd per wave, slots in lane order.
// Every lane of the wave must call it.
__device__ __forceinline__ int wave_append(int* counter, bool pred) {
    uint64_t mask = __ballot(pred);
    if (mask == 0) return -1;
    int leader = __ffsll((unsigned long long)mask) - 1;
    int base = 0;
    if (lane_id() == leader) base = atomicAdd(counter, __popcll(mask));
    base = __shfl(base, leader);
    int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    return pred ? base + rank : -1;
}

// Block-aggregated append: one atomicAdd per *block* (the queue counters are the contended words —
// one wave-level atomic per wave saturated a single counter, MI355X_MICROARCH "dequeue" ≈88/µs).
// Every thread of the block must call it (block-uniform control flow).
__device__ __forceinline__ int block_append(int* counter, bool pred, int* lds) {
    constexpr int NW = kBlock / 64;
    uint64_t mask = __ballot(pred);
    int wave = threadIdx.x >> 6;
    int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    if (lane_id() == 0) lds[wave] = __popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < NW; ++w) { int cw = lds[w]; lds[w] = tot; tot += cw; }
        lds[NW] = tot ? atomicAdd(counter, tot) : 0;
    }
    __syncthreads();
    int base = lds[NW] + lds[wave];
    __syncthreads();
    return pred ? base + rank : -1;
}

// Block-aggregated append of a static chunk's two items (kStaticItems = 2): one atomicAdd and one round of barriers
// for both; the block's first items take the lower positions, its second items the upper ones.  lds: 2 NW + 1 ints.
__device__ __forceinline__ void block_append2(int* counter, bool p0, bool p1, int* lds, int& o0, int& o1) {
    constexpr int NW = kBlock / 64;
    const uint64_t m0 = __ballot(p0), m1 = __ballot(p1);
    const int wave = threadIdx.x >> 6;
    const int r0 = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
    const int r1 = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
    if (lane_id() == 0) { lds[wave] = __popcll(m0); lds[NW + wave] = __popcll(m1); }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < 2 * NW; ++w) { int cw = lds[w]; lds[w] = tot; tot += cw; }
        lds[2 * NW] = tot ? atomicAdd(counter, tot) : 0;
    }
    __syncthreads();
    o0 = p0 ? lds[2 * NW] + lds[wave] + r0 : -1;
    o1 = p1 ? lds[2 * NW] + lds[NW + wave] + r1 : -1;
    __syncthreads();
}

// Work distribution of the persistent queue kernels over a sharded queue (rt_internal.h QueueView).
__device__ __forceinline__ int q_len(const QueueView& q, int j) {
    if (q.len) return q.len[j * kQStride];
    const int c = q.n - j * q.S;
    return c < 0 ? 0 : (c > q.S ? q.S : c);
}

// Static chunks (no tickets): the chunks of kStaticItems x kBlock items are interleaved over the shards (list entry
// 8c + j = chunk c of shard j) and block b takes entries b, b + grid, ... — with a grid that is a multiple of 8
// (resident grids are), a block stays on shard b % 8.  Every thread of the block walks the same entries.
static constexpr int kStaticItems = 2;  // items per thread per chunk (single-leaf scenes)
static constexpr int kChunk = kStaticItems * kBlock;
struct StaticChunks {
    QueueView q;
    int e, end;  // current list entry, list length
    int j, len;  // its shard and that shard's length
    __device__ __forceinline__ explicit StaticChunks(const QueueView& qv) : q(qv), e((int)blockIdx.x - (int)gridDim.x) {
        int mx = 0;
#pragma unroll
        for (int k = 0; k < kShards; ++k) {
            const int l = k < q.ns ? q_len(q, k) : 0;
            mx = l > mx ? l : mx;
        }
        end = q.ns * ((mx + kChunk - 1) / kChunk);
    }
    // next non-empty entry of this block: false when the list is done; chunk items are idx in [base, base + kChunk)
    __device__ __forceinline__ bool next(int& base) {
        while ((e += gridDim.x) < end) {
            j = e % q.ns;
            len = q_len(q, j);
            base = (e / q.ns) * kChunk;
            if (base < len) return true;
        }
        return false;
    }
};

// Wave tickets: a wave takes 64-item chunks of its preferred shard (blockIdx % 8) from that shard's ticket counter
// (the next ticket is requested while the current chunk runs), then drains the other shards in turn.  A shard whose
// ticket already passed its length is skipped without an atomic.
struct WaveTickets {
    int* tk;
    QueueView q;
    int j0, tries, j, len, pref;
    __device__ __forceinline__ int grab(int jj, int l) {
        int t = 0;
        if (lane_id() == 0 && l > 0) {
            t = __hip_atomic_load(tk + jj * kQStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t * 64 < l) t = atomicAdd(tk + jj * kQStride, 1);
        }
        return t;
    }
    __device__ __forceinline__ WaveTickets(int* t, const QueueView& qv) : tk(t), q(qv) {
        j0 = (int)(blockIdx.x % (unsigned)q.ns);
        tries = 0;
        j = j0;
        len = q_len(q, j);
        pref = grab(j, len);
    }
    // next chunk: shard jj, items idx in [base, min(base + 64, len)); false when every shard is drained
    __device__ __forceinline__ bool next(int& jj, int& base) {
        while (true) {
            const int t = __shfl(pref, 0);
            if (t * 64 < len) {
                jj = j;
                base = t * 64;
                if (lane_id() == 0) pref = atomicAdd(tk + j * kQStride, 1);
                return true;
            }
            if (++tries >= q.ns) return false;
            j = (j0 + tries) % q.ns;
            len = q_len(q, j);
            pref = grab(j, len);
        }
    }
};

// The items of a queue for kernels that append (every thread of the block, or of the wave, calls next() in step):
// WAVE = per-wave tickets (one item per lane per chunk), otherwise the block's static chunks (kStaticItems steps per
// chunk).  Yields the shard j, the index within it and whether this lane's item exists.
template <bool WAVE>
struct QueueItems;
template <>
struct QueueItems<true> {
    WaveTickets tk;
    __device__ __forceinline__ QueueItems(int* t, const QueueView& q) : tk(t, q) {}
    __device__ __forceinline__ bool next(int& j, int& idx, bool& live) {
        int base;
        if (!tk.next(j, base)) return false;
        idx = base + lane_id();
        live = idx < tk.len;
        return true;
    }
};
template <>
struct QueueItems<false> {
    StaticChunks ch;
    int base, r;
    __device__ __forceinline__ QueueItems(int*, const QueueView& q) : ch(q), base(0), r(kStaticItems) {}
    __device__ __forceinline__ bool next(int& j, int& idx, bool& live) {
        if (r >= kStaticItems) {
            if (!ch.next(base)) return false;
            r = 0;
        }
        j = ch.j;
        idx = base + r * kBlock + (int)threadIdx.x;
        ++r;
        live = idx < ch.len;
        return true;
    }
};

// One shard, static chunks (single-leaf scenes): block b takes chunks b, b + grid, ... of the queue's only shard.
struct QueueItemsOne {
    int n, c, r;
    __device__ __forceinline__ QueueItemsOne(int*, const QueueView& q)
        : n(q_len(q, 0)), c((int)blockIdx.x), r(0) {}
    __device__ __forceinline__ bool next(int& j, int& idx, bool& live) {
        if (r == kStaticItems) {
            r = 0;
            c += gridDim.x;
        }
        const int base = c * kChunk;
        if (base >= n) return false;
        j = 0;
        idx = base + r * kBlock + (int)threadIdx.x;
        ++r;
        live = idx < n;
        return true;
    }
};

// Append to the next queue: per wave (ticket kernels, no block-level synchronisation) or per block.
template <bool WAVE>
__device__ __forceinline__ int queue_append(int* counter, bool pred, int* lds) {
    if constexpr (WAVE) return wave_append(counter, pred);
    else return block_append(counter, pred, lds);
}


typedef unsigned long long ctr_t;
__device__ __forceinline__ void count_add(unsigned long long* ctr, int slot, unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int sub = (int)((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kCtrSubs - 1));
    if (lane_id() == 0 && v) atomicAdd(ctr + ctr_word(slot, sub), v);
}

__device__ __forceinline__ void sample_of(const SampleIds& ids, int s, int& pixel, int& index) {
    if (ids.ex_pixel) { pixel = ids.ex_pixel[s]; index = ids.ex_index[s]; return; }
    int i = ids.np_div.m ? intdiv(s, ids.np_div) : s / ids.n_pixels;
    int j = s - i * ids.n_pixels;
    pixel = ids.work_pixels[j];
    index = ids.index_begin + i;
}
// RayTracerTestApp.h:289-291 (raster y in [1, resY], a kept quirk)
__device__ __forceinline__ void pixel_xy(const DevFilm& film, int pixel, int& x, int& y) {
    if (film.rx_div.m) {
        const int q = intdiv(pixel, film.rx_div);
        x = pixel - q * film.res_x;
        y = film.y_int ? film.res_y - q : (int)((float)film.res_y - floorf((float)pixel / (float)film.res_x));
        return;
    }
    x = pixel % film.res_x;
    y = (int)((float)film.res_y - floorf((float)pixel / (float)film.res_x));
}

__device__ __forceinline__ void load8(const float4* a, const float4* b, int s, float v[8]) {
    float4 p = a[s], q = b[s];
    v[0] = p.x; v[1] = p.y; v[2] = p.z; v[3] = p.w; v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
}
__device__ __forceinline__ void load8_or_zero(const float4* a, const float4* b, int s, float v[8], bool zero) {
    if (zero) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 0.f;
    } else {
        load8(a, b, s, v);
    }
}
__device__ __forceinline__ void store8(float4* a, float4* b, int s, const float v[8]) {
    a[s] = make_float4(v[0], v[1], v[2], v[3]);
    b[s] = make_float4(v[4], v[5], v[6], v[7]);
}
// fields of a slot's path state (rt_internal.h RecView, R_*)
__device__ __forceinline__ float4* recf(const RecView& r, int slot, int f) {
    return r.p + (size_t)f * r.fs + (size_t)slot * r.ss;
}
__device__ __forceinline__ void rload8(const RecView& r, int slot, int f, float v[8]) {
    const float4* q = recf(r, slot, f);
    load8(q, q + r.fs, 0, v);
}
__device__ __forceinline__ void rload8_or_zero(const RecView& r, int slot, int f, float v[8], bool zero) {
    const float4* q = recf(r, slot, f);
    load8_or_zero(q, q + r.fs, 0, v, zero);
}
__device__ __forceinline__ void rstore8(const RecView& r, int slot, int f, const float v[8]) {
    float4* q = recf(r, slot, f);
    store8(q, q + r.fs, 0, v);
}
__device__ __forceinline__ uint2* rng8_state(const RecView& r) { return reinterpret_cast<uint2*>(r.p + R_RNG * r.fs); }
__device__ __forceinline__ float rec_prev_pdf(const RecView& r, int slot) { return recf(r, slot, R_MISC)->y; }
__device__ __forceinline__ void rec_set_prev_pdf(const RecView& r, int slot, float p) {
    reinterpret_cast<float*>(recf(r, slot, R_MISC))[1] = p;
}

// The wavelength warps' tables (rt_logtab.h: 97 log rows of 3 doubles, 64 exp rows of 2) staged in LDS by the
// kernels that evaluate the warps for every sample (k_generate: 8 atanh = 16 log rows; k_path_film: 8 cosh = 16
// exp rows): the rows are indexed per lane, so from the constant arrays each is a divergent vector-memory load.
__shared__ double g_logtab[rtm::kLogN][4];  // (row padded to 32 B: one ds_read_b128 + one ds_read_b64)
__shared__ double g_exptab[64][2];
struct WarpTabLds {
    __device__ static const double* logrow(int j) { return g_logtab[j]; }
    __device__ static const double* exprow(int j) { return g_exptab[j]; }
};
using WarpTab = WarpTabLds;
__device__ __forceinline__ void stage_warp_tables() {
    for (int i = threadIdx.x; i < rtm::kLogN * 3; i += blockDim.x) g_logtab[i / 3][i % 3] = rtm::kLogTab[i / 3][i % 3];
    for (int i = threadIdx.x; i < 64 * 2; i += blockDim.x) g_exptab[i / 2][i % 2] = rtm::kExp2Tab[i / 2][i % 2];
    __syncthreads();
}

// ===================================================================================== K1 generate
// RayTracerTestApp.h:305-323: StartPixelSample → SampleVisible(Get1D) → filter.Sample(GetPixel2D) →
// pixel + .5 + p → PerspectiveCamera::generateRay (Cameras.h:273-297) → Ray::Transform (Shapes.h:37-41).
// One camera sample of pixel (x, y): the sampler started at `index`, the 8 hero wavelengths and the world ray (w = 0).
__device__ __forceinline__ void camera_sample(const DevCamera& cam, const DevSampler& smp, const DevFilm& film, int x,
                                              int y, int index, Smp& sm, float lam[8], float4& ro, float4& rd) {
    sm.start(smp, x, y, index, 0);
    float u = sm.get1d(smp);
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // spectrum.h:322-336
        float up = u + float(i) / 8;
        if (up > 1) up -= 1;
        lam[i] = sample_visible_wavelength<WarpTab>(up);
    }
    float u0, u1;
    sm.get_pixel2d(smp, u0, u1);  // Sampler::GetPixel2D (RayTracerTestApp.h:316)
    float fx, fy;
    if (film.filter == 0) { fx = lerpf_(u0, -film.rx, film.rx); fy = lerpf_(u1, -film.ry, film.ry); }
    else if (film.filter == 1) { fx = sample_tent(u0, film.rx); fy = sample_tent(u1, film.ry); }
    else {  // Gaussian / Lanczos: tabulated inversion (filters.h:128-134, 239-245), weight f/pdf = 1
        fx = inversion_sample(film.cdf_x, film.cdf_n, -film.rx, film.rx, u0);
        fy = inversion_sample(film.cdf_y, film.cdf_n, -film.ry, film.ry, u1);
    }
    float posx = ((float)x + .5f) + fx, posy = ((float)y + .5f) + fy;
    V3 d, o;
    if (cam.type == 0) {  // PerspectiveCamera (Cameras.h:273-297)
        float np[4];
        mat4_mul(cam.r2c, posx, posy, 0.f, 1.f, np);
        d = vnorm(v3(np[0] / np[3], np[1] / np[3], np[2] / np[3]));
        o = v3(0, 0, 0);
        if (cam.lens_radius > 0) {
            float a0, a1, dx, dy;
            sm.get2d(smp, a0, a1);
            disk_concentric(a0, a1, dx, dy);
            float lx = cam.lens_radius * dx, ly = cam.lens_radius * dy;
            float ft = cam.focal_distance / d.z;
            V3 pf = vadd(o, vmul(d, ft));
            o = v3(lx, ly, 0);
            d = vnorm(vsub(pf, o));
        }
    } else if (cam.type == 1) {  // OrthographicCamera (Cameras.h:230-243)
        float cp[4];
        mat4_mul(cam.r2c, posx, posy, 0.f, 1.f, cp);
        o = v3(cp[0], cp[1], cp[2]);
        d = v3(0, 0, 1);
    } else {
        float s4[4];
        mat4_mul(cam.r2s, posx, posy, 0.f, 1.f, s4);
        V3 sp = v3(s4[0], s4[1], s4[2]);
        if (cam.type == 2) {  // PinholeCamera (Cameras.h:328-339): through the hole's centre
            o = sp;
            d = vnorm(vsub(v3(0.0f, 0.0f, cam.pinhole_depth), sp));
        } else {  // ThinlensCamera (Cameras.h:378-400), (lens_angle, len_percent_r) = (360 u0, u1)
            float a0, a1;
            sm.get2d(smp, a0, a1);
            float ang = (a0 * 360.0f) * 0.01745329251994329576923690768489f;
            float sn, cs;
            sincos_det(ang, sn, cs);
            float half = cam.thin_aperture / 2.0f;
            o = v3(a1 * half * cs, a1 * half * sn, cam.sensor_depth);
            V3 lc = v3(0, 0, cam.sensor_depth);
            V3 tmp = vnorm(vsub(lc, sp));
            float t = cam.thin_focal / tmp.z;
            V3 fpos = vadd(lc, vmul(tmp, t));
            d = vnorm(vsub(fpos, o));
        }
    }
    float wo[4], wd[4];
    mat4_mul(cam.c2w, o.x, o.y, o.z, 1.f, wo);
    mat4_mul(cam.c2w, d.x, d.y, d.z, 0.f, wd);
    float inv = 1.0f / sqrtf((wd[0] * wd[0] + wd[1] * wd[1]) + (wd[2] * wd[2] + wd[3] * wd[3]));  // glm dot vec4
    ro = make_float4(wo[0], wo[1], wo[2], 0.f);
    rd = make_float4(wd[0] * inv, wd[1] * inv, wd[2] * inv, 0.f);
}

// 4 waves/SIMD (158 -> 128 VGPRs, 112 B/lane spill): +3 % on the Cornell box.  The pdf streams are stored only in
// the reference mode (not lean); a lean instantiation without the pdf[8] registers (103 VGPRs, no spill) measured
// Cornell -0.9 % (round 4, two interleaved rounds), so one kernel serves both.
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) k_generate(int nS, SampleIds ids, DevCamera cam, DevSampler smp,
                                                     DevFilm film, GenOut out) {
    stage_warp_tables();
    if (out.zero)
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * kQRegion; i += gridDim.x * blockDim.x) out.zero[i] = 0;
    const bool with_pdf = !out.lean;
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nS; s += gridDim.x * blockDim.x) {
        int pixel, index, x, y;
        sample_of(ids, s, pixel, index);
        pixel_xy(film, pixel, x, y);
        Smp sm;
        float lam[8], pdf[8];
        float4 ro, rd;
        camera_sample(cam, smp, film, x, y, index, sm, lam, ro, rd);
#pragma unroll
        for (int i = 0; i < 8; ++i) pdf[i] = with_pdf ? visible_pdf<WarpTab>(lam[i]) : 0.f;
        // the origin's w carries the path slot (= s for camera rays) through every queue and sort
        out.rayO[s << out.rsh] = make_float4(ro.x, ro.y, ro.z, __int_as_float(s));
        out.rayD[s << out.rsh] = rd;
        if (with_pdf) store8(out.pdfA, out.pdfB, s, pdf);
        if (out.rec.p) {  // path mode: the slot's state
            rstore8(out.rec, s, R_LAM, lam);
            if (out.rec.rng8)
                rng8_state(out.rec)[s] = make_uint2((uint32_t)sm.rng.state, (uint32_t)(sm.rng.state >> 32));
            else
                *reinterpret_cast<uint4*>(recf(out.rec, s, R_RNG)) =  // (state, pixel id: restore_sampler)
                    make_uint4((uint32_t)sm.rng.state, (uint32_t)(sm.rng.state >> 32), (uint32_t)pixel, 0u);
            if (out.lean != 1)  // (dimension, prevPdf 0, TerminateSecondary flag 0)
                *recf(out.rec, s, R_MISC) = make_float4(__int_as_float(sm.dim), 0.f, 0.f, __int_as_float(pixel));
            if (!out.lean) {
                const float one[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
                const float zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                rstore8(out.rec, s, R_BETA, one);
                rstore8(out.rec, s, R_L, zero);
            }
        } else {
            store8(out.lamA, out.lamB, s, lam);
        }
    }
}

// Dense spectra in LDS (DevSpectra::SPK, {SR, SG, SB, D65} per nm, 7.5 KB): the hero wavelengths of a wave are spread
// over 360..830 nm, so a dense_query from global memory is a gather over ~15 cache lines per wave-instruction, and
// the sensor conversion makes 24 of them per sample; from LDS it is one ds_read_b128 per wavelength.  Same values,
// same index (spectrum.h:386-398: lround(λ) - 360, 0 outside the table), same arithmetic order: bit-identical.
__shared__ float4 g_spk[kSpecN];
__device__ __forceinline__ void stage_spectra(const DevSpectra* sp) {
    for (int i = threadIdx.x; i < kSpecN; i += blockDim.x) g_spk[i] = sp->SPK[i];
    __syncthreads();
}
__device__ __forceinline__ float4 spk_query(const DevSpectra* sp, float lambda) {
    long off = (long)roundf(lambda) - 360;  // std::lround: half away from zero
    if (off < 0 || off >= kSpecN) return make_float4(0.f, 0.f, 0.f, 0.f);
    return g_spk[off];
}
__device__ __forceinline__ float d65_query(const DevSpectra* sp, float lambda) { return spk_query(sp, lambda).w; }
// pixelsensor.h:81-87 (to_sensor_rgb, rt_device.h) over the staged table: per channel the same sum in the same order
__device__ __forceinline__ void to_sensor_rgb_spk(const DevSpectra* sp, const float L_[8], const float lam[8],
                                                  const float pdf[8], float ir, float rgb[3]) {
    float L[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) L[i] = (pdf[i] != 0) ? L_[i] / pdf[i] : 0.f;
    float4 q = spk_query(sp, lam[0]);
    float sr = q.x * L[0], sg = q.y * L[0], sb = q.z * L[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) {
        q = spk_query(sp, lam[i]);
        sr += q.x * L[i];
        sg += q.y * L[i];
        sb += q.z * L[i];
    }
    rgb[0] = ir * (sr / 8);
    rgb[1] = ir * (sg / 8);
    rgb[2] = ir * (sb / 8);
}

// Loads through the constant address space: with a wave-uniform index they become s_load (scalar cache).
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ldc4(const float4* p, int i) {
    f4v v = ((const __attribute__((address_space(4))) f4v*)p)[i];
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int2 ldc2i(const int2* p, int i) {
    i2v v = ((const __attribute__((address_space(4))) i2v*)p)[i];
    return make_int2(v.x, v.y);
}
// a whole record (shape, light) at a wave-uniform index through the scalar cache
template <class T>
__device__ __forceinline__ T ldconst(const T* p, int i) {
    static_assert(sizeof(T) % 4 == 0, "dword records");
    T r;
    const __attribute__((address_space(4))) int* src = (const __attribute__((address_space(4))) int*)(p + i);
    int* dst = (int*)&r;
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) dst[k] = src[k];
    return r;
}

// Any-hit (shadow) query on a multi-level octree, depth first.  With a fixed tMax every node box test and every
// triangle test has the same outcome whatever the order, the leaves reached through passing boxes are the same set,
// and the query only asks whether some tested triangle hits (Octtree_Model.h:66-127 with an early exit).  So a
// depth-first walk returns exactly the BFS's answer, but reaches an occluder after `depth` descents instead of
// after sweeping every level above it, and needs a stack of `depth` entries instead of a frontier-sized FIFO.
// Stack entry = (first node of a group << 8) | its children still to visit; LDS, one column per thread.
// Used by the shadow-queue kernel (k_path_shadow); inline callers keep the BFS, whose registers the shade kernels can
// spare (DFS inline: CFG3 144 -> 135, CFG4 111 -> 87 Msamples/s under the 4-wave budgets).
static constexpr int kDfsDepth = 16;
__shared__ unsigned g_dfs[kDfsDepth * kBlock];
template <int KZ>
__device__ __forceinline__ bool occluded_dfs(const DevScene& sc, int set, V3 o, V3 d, float tMax,
                                             ctr_t& nn, ctr_t& nt) {
    const V3 inv = v3(1 / d.x, 1 / d.y, 1 / d.z);
    const TriRay R = make_triray<KZ>(o, d);
    const int2* __restrict__ lr = sc.leafRange[set];
    const float4* __restrict__ tiles = sc.tiles[set];
    unsigned* stk = g_dfs + threadIdx.x;
    int sp = 0;
    int g = 0;          // first node of the current group (the root is a group of one)
    unsigned pm;        // its children still to visit whose box passes
    int Ch[8];          // their first children (-1: leaf), kept in registers for the current group
    int lf = 0, lc = 0; // pending leaf: first tile, triangle count
    ++nn;
    {
        const float4 a = sc.nodeA[0];
        pm = box_entry(a, sc.nodeB[0], o, inv) <= tMax ? 1u : 0u;
        Ch[0] = __float_as_int(a.w);
#pragma unroll
        for (int k = 1; k < 8; ++k) Ch[k] = -1;
    }
    bool done = false;
    while (true) {
        // node phase ("while-while", as the BFS): walk until this lane holds a non-empty leaf or runs out
        while (!done && lc == 0) {
            if (pm == 0) {
                if (sp == 0) { done = true; break; }
                const unsigned e = stk[--sp * kBlock];
                g = (int)(e >> 8);
                pm = e & 0xffu;
#pragma unroll
                for (int k = 0; k < 8; ++k) Ch[k] = __float_as_int(sc.nodeA[g + k].w);  // independent loads
                continue;
            }
            const int i = __builtin_ctz(pm);
            pm &= pm - 1;
            int child = Ch[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) child = i == k ? Ch[k] : child;
            if (child >= 0) {
                if (pm) stk[sp++ * kBlock] = ((unsigned)g << 8) | pm;
                g = child;
                float4 A8[8], B8[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) { A8[k] = sc.nodeA[g + k]; B8[k] = sc.nodeB[g + k]; }
                nn += 8;
                pm = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    pm |= (box_entry(A8[k], B8[k], o, inv) <= tMax ? 1u : 0u) << k;
                    Ch[k] = __float_as_int(A8[k].w);
                }
            } else {
                const int2 r = lr[g + i];
                lf = r.x;
                lc = r.y;
            }
        }
        if (lc == 0) return false;
        const int m = lc < kLeafChunk ? lc : kLeafChunk;
        for (int k = 0; k < m; ++k) {
            const float4* tp = tiles + 3 * (lf + k);
            ++nt;
            float b0, b1, b2, t;
            if (tri_intersect<KZ>(R, tMax, tp[0], tp[1], tp[2], b0, b1, b2, t) && t < tMax) return true;
        }
        lf += m;
        lc -= m;
    }
}

// Per-lane mask of the single-leaf culling clusters whose conservative box the ray reaches within tMax (bit c =
// cluster c, ncl <= 32).  The boxes are read through the scalar cache three clusters at a time, so a wave waits once
// per group instead of once per cluster (scalar loads return out of order: every use waits for all of them).
__device__ __forceinline__ uint32_t cluster_mask(const float4* cl, int ncl, bool far, V3 o, V3 inv, float tmax) {
    uint32_t hm = 0;
    for (int c0 = 0; c0 < ncl; c0 += 3) {
        float4 A[3], B[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int c = c0 + u < ncl ? c0 + u : ncl - 1;
            A[u] = ldc4(cl, 2 * c);
            B[u] = ldc4(cl, 2 * c + 1);
        }
#pragma unroll
        for (int u = 0; u < 3; ++u)
            if (c0 + u < ncl && (far || cluster_hit(A[u], B[u], o, inv, tmax))) hm |= 1u << (c0 + u);
    }
    return hm;
}
// triangles of the clusters in mask hm (the last cluster may hold fewer than kClusterTris of the leaf's n)
__device__ __forceinline__ int cluster_tris(uint32_t hm, int ncl, int n) {
    int t = __popc(hm) * kClusterTris;
    if ((hm >> (ncl - 1)) & 1u) t -= ncl * kClusterTris - n;
    return t;
}
// ===================================================================================== K2 traverse
// Octtree_Model.h:66-127 — FIFO BFS.  The 8 children of an internal node are contiguous, so the queue
// holds one entry per child *group*; popping a group visits its 8 nodes in order, which reproduces the
// reference's node-level FIFO order exactly.  tMax shrinks on every accepted hit ("t < tMax": the first
// hit found in BFS order wins ties), so hit ids, barycentrics and t are bit-identical to the reference's.
template <int QCAP, bool ANYHIT, int KZ, bool DFS = false>
__device__ __forceinline__ int traverse(const DevScene& sc, int set, V3 o, V3 d, float tMaxInit, float& rb0, float& rb1,
                                        float& rb2, float& rt, ctr_t& nn, ctr_t& nt) {
    V3 inv = v3(1 / d.x, 1 / d.y, 1 / d.z);
    TriRay R = make_triray<KZ>(o, d);
    float tMax = tMaxInit;
    int best = -1;
    const int2* __restrict__ lr = sc.leafRange[set];
    const float4* __restrict__ tiles = sc.tiles[set];
    if constexpr (QCAP == 1) {
        // The whole octree is one leaf (e.g. the 36-triangle Cornell box: 36 < TRIANGLE_CAPACITY): every
        // lane walks the same triangle list, so it is read through the scalar cache into SGPRs once per
        // wave; four triangles (12 x s_load_dwordx4) are fetched per scalar-cache round trip.
        ++nn;
        bool inside = box_hit(ldc4(sc.nodeA, 0), ldc4(sc.nodeB, 0), o, inv, tMax);
        int2 r = ldc2i(lr, 0);
        if (inside) {
            auto test = [&](float4 A, float4 B, float4 Cc) -> bool {
                ++nt;
                float b0, b1, b2, t;
                if (tri_intersect<KZ>(R, tMax, A, B, Cc, b0, b1, b2, t) && t < tMax) {
                    best = __float_as_int(Cc.y);
                    if (ANYHIT) return true;
                    tMax = t; rb0 = b0; rb1 = b1; rb2 = b2; rt = t;
                }
                return false;
            };
            constexpr int U = kTriUnroll;
            static_assert(U % 2 == 0, "pass 1 walks fan pairs");
            if (r.y <= 64) {
                // pass 1: every triangle's tMax-independent rejections (scalar-cache batches); pass 2: the full
                // test, in leaf order with the running tMax, on the survivors only — so the division and the
                // error-bound tail run per candidate, not once per triangle for whichever lane reached it
                uint64_t cand = 0;
                int k = 0;
                const uint64_t fp = sc.fan_pairs[set];  // bit k: leaf tiles k, k+1 share vertices (a,b,c),(a,c,d)
                // conservative cluster boxes first: a cluster no lane of the wave reaches is skipped whole
                // (closest hit: the box over [0, inf); any hit: over [0, tMax], exact for a fixed tMax).  Shadow rays
                // and coherent closest-hit waves (shared dominant axis: camera rays) cull by wave ballot; incoherent
                // closest-hit waves compact the passing (ray, cluster) pairs (culling every cluster: -2 %).
                const float4* cl = sc.clusters[set];
                const int ncl = sc.n_clusters[set];
                // (shadow rays compacted too: Cornell -7 % in r01, -6.5 % in r04)
                constexpr bool kCompact = !ANYHIT && KZ < 0;
                constexpr bool kCull = ANYHIT || KZ >= 0 || kCompact;
                const bool ncl_ok = ncl * kClusterTris >= r.y && ncl <= 32;  // the clusters cover the leaf
                auto far1 = [&](V3 p) {  // the pad is not sized for rays starting this far out: no cluster is skipped
                    const float gx = p.x - sc.cl_guard.x, gy = p.y - sc.cl_guard.y, gz = p.z - sc.cl_guard.z;
                    return gx * gx + gy * gy + gz * gz > sc.cl_guard.w;
                };
                if (kCull && ncl_ok) {
                    const float cl_t = ANYHIT ? tMax : 3.402823466e+38f;
                    const bool far = far1(o);
                    if (ANYHIT && kClusterTris == 2) {
                        // Shadow rays: each lane walks its own hit clusters, the tiles read from LDS (g_leaf1), so
                        // the wave runs as many candidate steps as its busiest lane has hit clusters instead of one
                        // per cluster any lane of the wave hit (Cornell bounce vertices: 0.75 hit clusters per shadow
                        // ray, but most of the 18 hit by some lane; r06_ab2: shade stage -10 %, Cornell +4.5 %).
                        // The candidate mask is exactly the per-cluster loop's, so pass 2 is unchanged.  Closest-hit
                        // bounce rays keep the compacted pairs below (this loop measured trace +8 % for them).
                        uint32_t hm = cluster_mask(cl, ncl, far, o, inv, cl_t);
                        nt += cluster_tris(hm, ncl, r.y);
                        while (hm) {
                            const int c = __builtin_ctz(hm);
                            hm &= hm - 1;
                            const float4* tp = RT_LEAF1(tiles, r.x, 2 * c);
                            unsigned bits;
                            if ((fp >> (2 * c)) & 1) {
                                bits = tri_candidate_pair<KZ>(R, tp[0], tp[1], tp[2], tp[4], tp[5]);
                            } else {
                                bits = tri_candidate<KZ>(R, tp[0], tp[1], tp[2]) ? 1u : 0u;
                                if (2 * c + 1 < r.y && tri_candidate<KZ>(R, tp[3], tp[4], tp[5])) bits |= 2u;
                            }
                            cand |= (uint64_t)bits << (2 * c);
                        }
                        k = r.y;
                    } else if (kCompact && kClusterTris == 2 && ncl <= kCompactMaxClusters) {
                        // Each lane box-tests every cluster against its own ray; the passing (lane, cluster) pairs
                        // are appended to the wave's LDS list in cluster order (ballot + mbcnt), and the active
                        // lanes then split the list evenly: lane j runs the candidate tests of pairs j, j + n, ...
                        // on the pair's ray (staged in LDS) and ORs the result bits into that ray's mask.  The
                        // per-(ray, triangle) test is unchanged, so the mask — and pass 2 — are exactly as before;
                        // only the SIMD no longer runs tests for lanes whose box missed (Cornell bounce rays: 2.7
                        // of 18 cluster boxes hit, but 17.7 of 18 hit by some lane of a wave).
                        CompactWave& cw = g_cmp[threadIdx.x >> 6];
                        const int ln = lane_id();
                        const uint64_t act = __ballot(true);
                        cw.ra[ln] = make_float4(R.Sx, R.Sy, R.Sz, R.ox);
                        cw.rb[ln] = make_float4(R.oy, R.oz, __int_as_float(R.kz), 0.f);
                        cw.cand[ln] = 0;
                        int np = 0;
                        const uint32_t hm = cluster_mask(cl, ncl, far, o, inv, cl_t);
                        nt += cluster_tris(hm, ncl, r.y);  // executed tests: the hit clusters' (the reference: all)
                        for (int c = 0; c < ncl; ++c) {
                            const bool hb = (hm >> c) & 1u;
                            uint64_t m = __ballot(hb);
                            if (hb) cw.pair[np + mbcnt64(m)] = (unsigned short)(ln | (c << 6));
                            np += __popcll(m);
                        }
                        wave_lds_sync();
                        const int nact = __popcll(act);
                        for (int p = mbcnt64(act); p < np; p += nact) {
                            const unsigned v = cw.pair[p];
                            const int L = v & 63, c = v >> 6;
                            const float4 ra = cw.ra[L], rb = cw.rb[L];
                            TriRay Q;
                            Q.Sx = ra.x; Q.Sy = ra.y; Q.Sz = ra.z; Q.ox = ra.w; Q.oy = rb.x; Q.oz = rb.y;
                            Q.kz = KZ >= 0 ? KZ : __float_as_int(rb.z);
                            Q.kx = Q.kz + 1; if (Q.kx == 3) Q.kx = 0;
                            Q.ky = Q.kx + 1; if (Q.ky == 3) Q.ky = 0;
                            const float4* tp = RT_LEAF1(tiles, r.x, 2 * c);
                            unsigned bits;
                            if ((fp >> (2 * c)) & 1) {
                                bits = tri_candidate_pair<KZ>(Q, tp[0], tp[1], tp[2], tp[4], tp[5]);
                            } else {
                                bits = tri_candidate<KZ>(Q, tp[0], tp[1], tp[2]) ? 1u : 0u;
                                if (2 * c + 1 < r.y && tri_candidate<KZ>(Q, tp[3], tp[4], tp[5])) bits |= 2u;
                            }
                            if (bits) atomicOr(&cw.cand[L], (unsigned long long)bits << (2 * c));
                        }
                        wave_lds_sync();
                        cand = cw.cand[ln];
                        k = r.y;
                    } else {
                    const uint32_t hm = cluster_mask(cl, ncl, far, o, inv, cl_t);
                    nt += cluster_tris(hm, ncl, r.y);  // executed tests: the hit clusters' (the reference: all)
                    for (int c = 0; c < ncl; ++c) {
                        const bool hb = (hm >> c) & 1u;
                        if (__ballot(hb) == 0) continue;
                        if (kClusterTris == 2 && ((fp >> (2 * c)) & 1)) {
                            int e = 3 * (r.x + 2 * c);
                            if (hb)
                                cand |= (uint64_t)tri_candidate_pair<KZ>(R, ldc4(tiles, e), ldc4(tiles, e + 1),
                                                                         ldc4(tiles, e + 2), ldc4(tiles, e + 4),
                                                                         ldc4(tiles, e + 5)) << (2 * c);
                            continue;
                        }
#pragma unroll
                        for (int u = 0; u < kClusterTris; ++u) {
                            int kk = c * kClusterTris + u;
                            if (kk >= r.y) break;
                            int e = 3 * (r.x + kk);
                            if (hb && tri_candidate<KZ>(R, ldc4(tiles, e), ldc4(tiles, e + 1), ldc4(tiles, e + 2)))
                                cand |= 1ull << kk;
                        }
                    }
                    k = r.y;
                    }
                }
                nt += r.y - k;  // unculled: every triangle's candidate test runs
                for (; k + U <= r.y; k += U) {
                    int e = 3 * (r.x + k);
                    float4 T[3 * U];
#pragma unroll
                    for (int j = 0; j < 3 * U; ++j) T[j] = ldc4(tiles, e + j);
#pragma unroll
                    for (int u = 0; u < U; u += 2) {
                        if ((fp >> (k + u)) & 1) {  // wave-uniform: a scalar branch
                            cand |= (uint64_t)tri_candidate_pair<KZ>(R, T[3 * u], T[3 * u + 1], T[3 * u + 2],
                                                                     T[3 * u + 4], T[3 * u + 5]) << (k + u);
                        } else {
                            if (tri_candidate<KZ>(R, T[3 * u], T[3 * u + 1], T[3 * u + 2])) cand |= 1ull << (k + u);
                            if (tri_candidate<KZ>(R, T[3 * u + 3], T[3 * u + 4], T[3 * u + 5]))
                                cand |= 1ull << (k + u + 1);
                        }
                    }
                }
                for (; k < r.y; ++k) {
                    int e = 3 * (r.x + k);
                    if (tri_candidate<KZ>(R, ldc4(tiles, e), ldc4(tiles, e + 1), ldc4(tiles, e + 2))) cand |= 1ull << k;
                }
                // Closest hit, nearest cluster first (the canonical rule of §6b on the single leaf).  The leaf-order
                // pass below tests every candidate; here a lane tests the candidate cluster its ray enters first,
                // then only the clusters entered within cut = t1 + 2 W(t1), and keeps the two smallest t.  If the
                // runner-up lies beyond t1 + W(t1) the leaf-order pass must end on t1's triangle with the same
                // (b, t): it is accepted robustly whatever hit came before it, and no later hit can be accepted.
                // The skipped clusters' triangles lie beyond their padded boxes' entry, so beyond t1 + W.  Near
                // ties (shared edges, coplanar faces) fall through to the exact leaf-order pass.
                if (!ANYHIT && kClusterTris == 2 && cand && ncl_ok) {
                    const bool far_o = far1(o);
                    auto entry = [&](int c) {
                        if (far_o) return 0.f;
                        const float4 A = g_cl1[2 * c], B = g_cl1[2 * c + 1];
                        const float x0 = (A.x - o.x) * inv.x, x1 = (B.x - o.x) * inv.x;
                        const float y0 = (A.y - o.y) * inv.y, y1 = (B.y - o.y) * inv.y;
                        const float z0 = (A.z - o.z) * inv.z, z1 = (B.z - o.z) * inv.z;
                        return fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.f));
                    };
                    float t1 = __builtin_inff(), t2 = __builtin_inff(), cut = __builtin_inff();
                    int w1 = -1;
                    float c0 = 0.f, c1 = 0.f, c2 = 0.f;
                    auto test_cluster = [&](int c) {
                        uint32_t bits = (uint32_t)(cand >> (2 * c)) & 3u;
                        while (bits) {
                            const int j = 2 * c + __builtin_ctz(bits);
                            bits &= bits - 1;
                            const float4* tp = RT_LEAF1(tiles, r.x, j);
                            float b0, b1, b2, t;
                            if (tri_intersect<KZ>(R, tMaxInit, tp[0], tp[1], tp[2], b0, b1, b2, t) && t < tMaxInit) {
                                if (t < t1) {
                                    t2 = t1; t1 = t; w1 = j; c0 = b0; c1 = b1; c2 = b2;
                                    cut = t1 + 2.f * (t1 * 0x1p-16f + sc.wabs);
                                } else if (t < t2) {
                                    t2 = t;
                                }
                            }
                        }
                    };
                    uint64_t cm = (cand | (cand >> 1)) & 0x5555555555555555ull;  // bit 2c: cluster c has candidates
                    int cn = -1;
                    float en = __builtin_inff();
                    for (uint64_t m = cm; m; m &= m - 1) {
                        const int c = __builtin_ctzll(m) >> 1;
                        const float e = entry(c);
                        if (e < en || cn < 0) { en = e; cn = c; }
                    }
                    test_cluster(cn);
                    cm &= ~(1ull << (2 * cn));
                    for (; cm; cm &= cm - 1) {
                        const int c = __builtin_ctzll(cm) >> 1;
                        if (!(entry(c) > cut)) test_cluster(c);
                    }
                    if (!(t2 <= t1 + (t1 * 0x1p-16f + sc.wabs))) {  // decided (t1 = inf: no hit at all)
                        if (w1 >= 0) {
                            rb0 = c0; rb1 = c1; rb2 = c2; rt = t1;
                            return __float_as_int(RT_LEAF1(tiles, r.x, w1)[2].y);
                        }
                        return -1;
                    }
                }
                while (cand) {
                    int j = __builtin_ctzll(cand);
                    cand &= cand - 1;
                    const float4* tp = RT_LEAF1(tiles, r.x, j);
                    float b0, b1, b2, t;
                    if (tri_intersect<KZ>(R, tMax, tp[0], tp[1], tp[2], b0, b1, b2, t) && t < tMax) {
                        best = __float_as_int(tp[2].y);
                        if (ANYHIT) return best;
                        tMax = t; rb0 = b0; rb1 = b1; rb2 = b2; rt = t;
                    }
                }
                return best;
            }
            int k = 0;
            for (; k + U <= r.y; k += U) {
                int e = 3 * (r.x + k);
                float4 T[3 * U];
#pragma unroll
                for (int j = 0; j < 3 * U; ++j) T[j] = ldc4(tiles, e + j);
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (test(T[3 * u], T[3 * u + 1], T[3 * u + 2]) && ANYHIT) return best;
            }
            for (; k < r.y; ++k) {
                int e = 3 * (r.x + k);
                if (test(ldc4(tiles, e), ldc4(tiles, e + 1), ldc4(tiles, e + 2)) && ANYHIT) return best;
            }
        }
        return best;
    }
    if constexpr (ANYHIT && DFS) {
        if (sc.depth <= kDfsDepth)  // the upload's octree depth; deeper trees keep the BFS FIFO below
            return occluded_dfs<KZ>(sc, set, o, d, tMax, nn, nt) ? 0 : -1;  // any-hit: 0 = occluded
    }
    // Group FIFO.  QCAP > 1: a private array (registers) holding the host's exact worst-case bound.
    // QCAP == 0: the first kLdsQ entries of each lane's FIFO live in LDS as 16-bit group ids (first child =
    // 8 g + 1); once a push finds them full the lane spills every later push to its HBM ring (sized by the
    // bound) until the FIFO drains, so pops read LDS for positions below `spill` and HBM from there on.
    constexpr bool GQ = QCAP == 0;
    int q[GQ ? 1 : QCAP];
    // the FIFO lives in this thread's own column of the BVH stacks (waves of the block may still be walking theirs):
    // entry j at 16-bit word (j / 4) * 4 kBlock + j % 4 of the column
    unsigned short* lq = reinterpret_cast<unsigned short*>(g_bstk + threadIdx.x);
    int* gq = GQ ? sc.ring + (blockIdx.x * blockDim.x + threadIdx.x) : nullptr;
    const int qmask = GQ ? sc.ring_mask : QCAP - 1;
    int spill = 0x7fffffff;
    int head = 0, tail = 0;
    bool done = false;
    int lf = 0, lc = 0;  // pending leaf: first tile, triangle count
    // The 8 children of a popped group are fetched together (16 independent float4 loads) and reduced to
    // entry distances E[i] (box_entry: the box test passes for tMax iff E[i] <= tMax); the visit mask is
    // re-evaluated whenever a leaf has shrunk tMax, so every child is still tested against the tMax the
    // reference's node-by-node BFS would use at that point.
    // "while-while" (Aila & Laine 2009): each lane walks its BFS until it reaches a non-empty leaf (or drains),
    // then the wave tests the pending leaves together.  A lane's own sequence of box and triangle tests — and
    // the tMax each sees — is unchanged, so results are the reference's bit for bit.
    int gfirst = 0;          // node index of child 0 of the current group
    unsigned pm;             // children still to visit whose box passes
    float E[8];
    int Ch[8];
    {
        float4 a = sc.nodeA[0], b = sc.nodeB[0];  // the root: a group of one
        ++nn;
        E[0] = box_entry(a, b, o, inv);
        Ch[0] = __float_as_int(a.w);
#pragma unroll
        for (int i = 1; i < 8; ++i) { E[i] = __builtin_inff(); Ch[i] = -1; }
        pm = E[0] <= tMax ? 1u : 0u;
    }
    while (true) {
        while (!done && lc == 0) {
            if (pm == 0) {
                if (head == tail) { done = true; break; }
                if constexpr (GQ) {
                    if (head < spill) {
                        const int j = head & (kLdsQ - 1);
                        gfirst = 8 * (int)lq[(j >> 2) * (4 * kBlock) + (j & 3)] + 1;
                    }
                    else gfirst = gq[(size_t)(head & qmask) * sc.ring_threads];
                } else {
                    gfirst = q[head & qmask];
                }
                ++head;
                if (GQ && head == tail) spill = 0x7fffffff;  // drained: LDS again
                nn += 8;
                pm = 0;
                {  // the 8 children's boxes in flight at once (4 or 2 at a time: fewer spills, CFG3 -4 %)
                    float4 A8[8], B8[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        A8[i] = sc.nodeA[gfirst + i];
                        B8[i] = sc.nodeB[gfirst + i];
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        E[i] = box_entry(A8[i], B8[i], o, inv);
                        Ch[i] = __float_as_int(A8[i].w);
                        pm |= (E[i] <= tMax ? 1u : 0u) << i;
                    }
                }
                continue;
            }
            int i = __builtin_ctz(pm);
            pm &= pm - 1;
            int child = Ch[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) child = i == k ? Ch[k] : child;
            if (child >= 0) {
                if constexpr (GQ) {
                    if (spill == 0x7fffffff && tail - head < kLdsQ) {
                        const int j = tail & (kLdsQ - 1);
                        lq[(j >> 2) * (4 * kBlock) + (j & 3)] = (unsigned short)((child - 1) >> 3);
                    } else {
                        if (spill == 0x7fffffff) spill = tail;
                        gq[(size_t)(tail & qmask) * sc.ring_threads] = child;
                    }
                } else {
                    q[tail & qmask] = child;
                }
                ++tail;
            } else {
                int2 r = lr[gfirst + i];
                lf = r.x;
                lc = r.y;
            }
        }
        if (lc == 0) break;
        // at most kLeafChunk triangles per phase: a lane in a big leaf (the CFG3 octree has leaves of up to 583
        // triangles) keeps the rest pending while the other lanes walk on to their next leaf
        int m = lc < kLeafChunk ? lc : kLeafChunk;
        // closest hit: software-pipelined leaf loop (the next triangle's 48 B in flight during a test; any-hit
        // callers keep the plain loop, whose registers the shade kernels cannot spare)
        constexpr bool PF = !ANYHIT;
        float4 nA, nB, nC;
        if constexpr (PF) { nA = tiles[3 * lf]; nB = tiles[3 * lf + 1]; nC = tiles[3 * lf + 2]; }
        for (int k = 0; k < m; ++k) {
            float4 A, B, Cc;
            if constexpr (PF) {
                A = nA; B = nB; Cc = nC;  // the next triangle's loads are issued before this one's test
                if (k + 1 < m) {
                    const float4* np = tiles + 3 * (lf + k + 1);
                    nA = np[0]; nB = np[1]; nC = np[2];
                }
            } else {
                const float4* tp = tiles + 3 * (lf + k);
                A = tp[0]; B = tp[1]; Cc = tp[2];
            }
            ++nt;
            float b0, b1, b2, t;
            if (tri_intersect<KZ>(R, tMax, A, B, Cc, b0, b1, b2, t) && t < tMax) {
                best = __float_as_int(Cc.y);
                if (ANYHIT) return best;
                tMax = t; rb0 = b0; rb1 = b1; rb2 = b2; rt = t;
            }
        }
        lf += m;
        lc -= m;
        if (lc > 0) continue;
        unsigned keep = 0;  // tMax may have shrunk: the remaining children are tested against the new value
#pragma unroll
        for (int k = 0; k < 8; ++k) keep |= (E[k] <= tMax ? 1u : 0u) << k;
        pm &= keep;
    }
    return best;
}

// The reference BFS (Octtree_Model.h:66-127) for ONE ray, run by a whole wave (every lane holds the same ray; all 64
// lanes active).  Used for the rays the BVH's canonical rule leaves ambiguous, in the kernel that
// found them: a lane's own BFS of such a ray tests ~300-600 boxes and ~500-1700 triangles one after the other (CPU
// counts over 11.6 M rays), a single-lane chain of dependent loads of about a millisecond, and it holds 147 VGPRs.
// Here the lanes split the work while the decisions stay exactly the node-by-node BFS's:
//   - a popped group's 8 child boxes are loaded and tested by lanes 0-7 against the tMax of that moment, then visited in
//     child order; a child whose box passed is re-tested when a leaf has shrunk tMax meanwhile (the BFS tests child k
//     after the leaves of children < k), so each box test sees the BFS's tMax;
//   - a leaf's triangles are tested 64 at a time against the tMax at the start of the batch, and the ones that pass
//     are tested again, in leaf order, with the running tMax — the BFS's own test sequence, since a triangle (or box)
//     that fails with some tMax fails with every smaller one (both tests are monotone in tMax; the canonical rule
//     rests on the same property), so the skipped tests are exactly failing ones;
//   - ANY (shadow rays, fixed tMax): occluded iff some reachable leaf has a passing triangle — the first one found
//     ends the search, as it ends the BFS;
//   - the FIFO holds 16-bit group ids (first child = 1 + 8 g) in the wave's own columns of an LDS stack array (its
//     walks are over; other waves of the block may still be walking in theirs): kCoopFifo entries.
// Returns false if the FIFO would overflow; the host launches no fallback kernel when the octree's exact worst-case
// queue fits (DevScene coop_ok), so a false return then never happens.
struct CoopFifo {
    unsigned short* base;  // the wave's row 0
    int row_stride;        // 16-bit words between rows
    int shift;             // log2 of the wave's 16-bit words per row
    __device__ __forceinline__ unsigned short& at(int e) const {
        e &= kCoopFifo - 1;
        return base[(e >> shift) * row_stride + (e & ((1 << shift) - 1))];
    }
};
static_assert(kBvhStack * 256 >= kCoopFifo && kAnyStack * 128 >= kCoopFifo && (kCoopFifo & (kCoopFifo - 1)) == 0,
              "the cooperative BFS FIFO fits the wave's stack columns");
__device__ __forceinline__ CoopFifo coop_fifo_bstk() {  // g_bstk: uint2 per (row, thread)
    return CoopFifo{reinterpret_cast<unsigned short*>(g_bstk) + 4 * (threadIdx.x & ~63u), 4 * kBlock, 8};
}
__device__ __forceinline__ CoopFifo coop_fifo_astk() {  // g_astk: unsigned per (row, thread)
    return CoopFifo{reinterpret_cast<unsigned short*>(g_astk) + 2 * (threadIdx.x & ~63u), 2 * kBlock, 7};
}
template <bool ANY>
__device__ __forceinline__ bool bfs_coop(const DevScene& sc, int set, V3 o, V3 d, float tMaxInit, const CoopFifo& Q,
                                         int& rprim, float& rb0, float& rb1, float& rb2, float& rt, ctr_t& nn,
                                         ctr_t& nt) {
    const int ln = lane_id();
    const V3 inv = v3(1 / d.x, 1 / d.y, 1 / d.z);
    const TriRay R = make_triray<-1>(o, d);
    const int2* __restrict__ lr = sc.leafRange[set];
    const float4* __restrict__ tiles = sc.tiles[set];
    float tMax = tMaxInit;
    int best = -1;
    int head = 0, tail = 0;
    ctr_t cn = 0, ct = 0;
    bool found = false;  // ANY: an occluder
    auto leaf = [&](int lf, int lc) {
        for (int base = 0; base < lc && !found; base += 64) {
            const int k = base + ln;
            bool c = false;
            float b0, b1, b2, t;
            if (k < lc) {
                const float4* tp = tiles + 3 * (lf + k);
                c = tri_intersect<-1>(R, tMax, tp[0], tp[1], tp[2], b0, b1, b2, t) && t < tMax;
            }
            uint64_t m = __ballot(c);
            if constexpr (ANY) {
                if (m) {
                    found = true;
                    best = __shfl(c ? __float_as_int(tiles[3 * (lf + k) + 2].y) : 0, __builtin_ctzll(m));
                }
            } else {
                while (m) {  // the candidates in leaf order, with the running tMax (uniform: every lane the same test)
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const float4* tp = tiles + 3 * (lf + base + l);
                    const float4 A = tp[0], B = tp[1], Cc = tp[2];
                    if (tri_intersect<-1>(R, tMax, A, B, Cc, b0, b1, b2, t) && t < tMax) {
                        best = __float_as_int(Cc.y);
                        tMax = t; rb0 = b0; rb1 = b1; rb2 = b2; rt = t;
                    }
                }
            }
        }
        ct += lc;
    };
    bool ok = true;
    {  // the root: a group of one
        const float4 a = sc.nodeA[0], b = sc.nodeB[0];
        ++cn;
        if (box_entry(a, b, o, inv) <= tMax) {
            const int ch = __float_as_int(a.w);
            if (ch >= 0) {
                if (ln == 0) Q.at(tail) = (unsigned short)((ch - 1) >> 3);
                ++tail;
            } else {
                const int2 r = lr[0];
                if (r.y) leaf(r.x, r.y);
            }
        }
    }
    while (head < tail && !found) {
        wave_lds_sync();
        const int g = 8 * (int)Q.at(head) + 1;
        ++head;
        float e = __builtin_inff();
        int ch = -1;
        if (ln < 8) {
            const float4 a = sc.nodeA[g + ln], b = sc.nodeB[g + ln];
            e = box_entry(a, b, o, inv);
            ch = __float_as_int(a.w);
        }
        cn += 8;
        unsigned pm = (unsigned)__ballot(ln < 8 && e <= tMax);
        while (pm && !found) {
            const int i = __builtin_ctz(pm);
            pm &= pm - 1;
            const float ei = __shfl(e, i);
            const int ci = __shfl(ch, i);
            if (!ANY && !(ei <= tMax)) continue;  // a leaf shrank tMax since the ballot
            if (ci >= 0) {
                if (tail - head >= kCoopFifo) { ok = false; break; }
                if (ln == 0) Q.at(tail) = (unsigned short)((ci - 1) >> 3);
                ++tail;
            } else {
                const int2 r = lr[g + i];
                if (r.y) leaf(r.x, r.y);
            }
        }
        if (!ok) break;
    }
    wave_lds_sync();  // (the FIFO's LDS is the walks' stacks: the wave's next walks write it)
    rprim = best;
    nn += cn;
    nt += ct;
    return ok;
}

// ============================================================= fast multi-level traversal
// The reference's unordered BFS (Octtree_Model.h:66-127) only shrinks tMax when its order happens to reach the
// near leaf, and its answer depends on that order only through near-ties.  Multi-level scenes therefore walk an
// 8-wide compressed BVH (rt_bvh.cpp) nearest-child first and apply the canonical rule of oracle/rtcore.hpp
// (Octree::ClosestCanonical / OccludedCanonical), which tests/test_canonical_traversal.py checks against the BFS
// on >= 10 M rays (over this BVH: oracle Bvh8Walk restates this walk bit for bit):
//   closest hit: keep the two smallest-t distinct triangles (t1, t2), prune with cut = t1 + 2 W(t1).  If
//                t2 > t1 + W(t1) the BFS must end on t1's triangle with the same (b, t); otherwise (or on a stack
//                overflow, or an origin beyond the guard) the ray is ambiguous;
//   any hit:     a passing triangle with t < tMax - W(tMax) proves occlusion; hits only inside the window are
//                ambiguous.
// Ambiguous rays — rare: coplanar / touching surfaces, near-tMax occluders — run the reference BFS.
__device__ __forceinline__ float canon_window(float t, float wabs) { return t * 0x1p-16f + wabs; }

// inv = 1 / d with |d| clamped to >= 2^-80: a zero component then gives huge but finite plane distances of the
// right sign (no inf - inf), and the clamped ray leaves a slab it starts in only after ~pad / 2^-80, far beyond any
// distance in a scene.
__device__ __forceinline__ V3 bvh_inv(V3 d) {
    const float e = 0x1p-80f;
    return v3(1 / copysignf(fmaxf(fabsf(d.x), e), d.x), 1 / copysignf(fmaxf(fabsf(d.y), e), d.y),
              1 / copysignf(fmaxf(fabsf(d.z), e), d.z));
}
// Rays the BVH may not decide: an origin beyond the padding's validity, or picked by the RTMI_FORCE_AMB test knob.
__device__ __forceinline__ bool bvh_refuses(const DevScene& sc, V3 o, V3 d) {
    if (!(fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)) <= sc.oguard)) return true;
    return sc.amb_force &&
           (((__float_as_uint(d.x) ^ (__float_as_uint(d.y) >> 3) ^ (__float_as_uint(d.z) >> 7)) & sc.amb_mask) == 0);
}
__device__ __forceinline__ void decode_leaf(int w, int& lf, int& lc) {
    lf = (w >> 4) & 0x7ffffff;
    lc = (w & 15) + 1;
}
__device__ __forceinline__ void kswap(unsigned& a, unsigned& b) {
    const unsigned lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo; b = hi;
}
static constexpr unsigned kNoChild = 0xffffffffu;
// Four consecutive floats at a 4-byte aligned address (the BVH's packed 36-B triangle tiles): one global_load_dwordx4
typedef float rt_f4u __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ float4 ld_f4u(const float* p) {
    const rt_f4u v = *reinterpret_cast<const rt_f4u*>(p);
    return make_float4(v.x, v.y, v.z, v.w);
}
static constexpr int kLeafStep = 8;  // triangles per leaf phase of the BVH walk (a held leaf's rest stays held)

// One 8-wide node against the ray: the sorted child keys k[0] <= ... <= k[7].  Key of a child whose slab interval
// [tn, tf] is non-empty within [0, tcut]: (bits(tn) with the low 3 bits cleared) | slot — tn >= 0, so the keys
// order the children by entry distance (truncated: a smaller value, the cull on pop stays conservative); missed
// and unused slots: kNoChild.  The slab test: the child's plane along axis a is origin_a + q 2^(e_a - 127), its
// parametric distance (plane - o_a) inv_a is evaluated as fma(q, inv_a 2^(e_a - 127), fma(origin_a, inv_a,
// -o_a inv_a)) — the scaling by a power of two is exact, so each plane moves by a few ulp of max(|o|, M) at
// most, which the build's padding covers (rt_host.cpp scene_bvh).  The near plane along a is the lo plane when
// inv_a >= 0, else the hi plane (the same interval as min / max of the two); tf is widened by 1.00000048 as the
// reference's IntersectP widens tFar (Shapes.h:116, 1 + 2 gamma(3)).
struct Bvh8Ray {
    V3 inv, oi;
};
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void node_keys(const BvhNode8& n, const Bvh8Ray& r, float tcut, unsigned k[8], bool sort) {
    const unsigned w0 = __float_as_uint(n.N0.w);
    const float sx = ldexpf(r.inv.x, (int)(w0 & 255u) - 127), sy = ldexpf(r.inv.y, (int)((w0 >> 8) & 255u) - 127),
                sz = ldexpf(r.inv.z, (int)((w0 >> 16) & 255u) - 127);
    const float bx = __builtin_fmaf(n.N0.x, r.inv.x, -r.oi.x), by = __builtin_fmaf(n.N0.y, r.inv.y, -r.oi.y),
                bz = __builtin_fmaf(n.N0.z, r.inv.z, -r.oi.z);
    const bool px = r.inv.x >= 0.f, py = r.inv.y >= 0.f, pz = r.inv.z >= 0.f;
    const unsigned nx0 = px ? n.QX.x : n.QX.z, nx1 = px ? n.QX.y : n.QX.w, fx0 = px ? n.QX.z : n.QX.x, fx1 = px ? n.QX.w : n.QX.y;
    const unsigned ny0 = py ? n.QY.x : n.QY.z, ny1 = py ? n.QY.y : n.QY.w, fy0 = py ? n.QY.z : n.QY.x, fy1 = py ? n.QY.w : n.QY.y;
    const unsigned nz0 = pz ? n.QZ.x : n.QZ.z, nz1 = pz ? n.QZ.y : n.QZ.w, fz0 = pz ? n.QZ.z : n.QZ.x, fz1 = pz ? n.QZ.w : n.QZ.y;
    const unsigned valid = n.N1.w;
    // (near, far) plane pairs of one axis in one packed FMA (v_pk_fma_f32: two IEEE fmas, the same bits)
    const f2v SX = {sx, sx}, SY = {sy, sy}, SZ = {sz, sz}, BX = {bx, bx}, BY = {by, by}, BZ = {bz, bz};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int sh = 8 * (s & 3);
        const unsigned nx = s < 4 ? nx0 : nx1, fx = s < 4 ? fx0 : fx1, ny = s < 4 ? ny0 : ny1, fy = s < 4 ? fy0 : fy1;
        const unsigned nz = s < 4 ? nz0 : nz1, fz = s < 4 ? fz0 : fz1;
        const f2v tx = __builtin_elementwise_fma((f2v){(float)((nx >> sh) & 255u), (float)((fx >> sh) & 255u)}, SX, BX);
        const f2v ty = __builtin_elementwise_fma((f2v){(float)((ny >> sh) & 255u), (float)((fy >> sh) & 255u)}, SY, BY);
        const f2v tz = __builtin_elementwise_fma((f2v){(float)((nz >> sh) & 255u), (float)((fz >> sh) & 255u)}, SZ, BZ);
        const float tn = fmaxf(fmaxf(tx.x, ty.x), fmaxf(tz.x, 0.f));
        const float tf = fminf(fminf(tx.y, ty.y), fminf(tz.y, tcut)) * 1.00000048f;
        k[s] = (((valid >> s) & 1u) && tn <= tf) ? ((__float_as_uint(tn) & 0x7ffffff8u) | (unsigned)s) : kNoChild;
    }
    if (!sort) return;  // (any-hit walks: any order gives the same answer)
    // Batcher's odd-even merge sort, 19 compare-exchanges
    kswap(k[0], k[1]); kswap(k[2], k[3]); kswap(k[4], k[5]); kswap(k[6], k[7]);
    kswap(k[0], k[2]); kswap(k[1], k[3]); kswap(k[4], k[6]); kswap(k[5], k[7]);
    kswap(k[1], k[2]); kswap(k[5], k[6]);
    kswap(k[0], k[4]); kswap(k[1], k[5]); kswap(k[2], k[6]); kswap(k[3], k[7]);
    kswap(k[2], k[4]); kswap(k[3], k[5]);
    kswap(k[1], k[2]); kswap(k[3], k[4]); kswap(k[5], k[6]);
}
// The child word of slot (key & 7): >= 0 an internal node, else a leaf 0x80000000 | first_tile << 4 | (count - 1)
__device__ __forceinline__ int child_word(const BvhNode8& n, unsigned key) {
    const unsigned s = key & 7u;
    const unsigned imask = __float_as_uint(n.N0.w) >> 24;
    const unsigned below = (1u << s) - 1u;
    if ((imask >> s) & 1u) return (int)(n.N1.x + (unsigned)__popc(imask & below));
    const unsigned cnt = (n.N1.z >> (4 * s)) & 15u;
    unsigned m = n.N1.z & ((1u << (4 * s)) - 1u);  // s <= 7: shift <= 28
    m = (m & 0x0f0f0f0fu) + ((m >> 4) & 0x0f0f0f0fu);
    const unsigned first = n.N1.y + ((m * 0x01010101u) >> 24);
    return (int)(0x80000000u | first << 4 | (cnt - 1u));
}

// The walk shared by both queries: nearest child first, the others pushed far-to-near on a per-lane LDS stack of
// (child word, key) (an entry whose entry distance lies beyond the current cut is dropped when popped); leaves are
// handed to `leaf(lf, lc)`, which may lower the cut and returns true to end the walk.  Returns false on a stack
// overflow (the ray is then ambiguous).
// ANY (any-hit, fixed cut): the entries are the child words alone on g_astk — every pushed child was entered within
// the fixed tMax, so there is nothing to cull on pop.
template <bool ANY, class LeafFn>
__device__ __forceinline__ bool bvh8_walk(const float4* __restrict__ nodes, const Bvh8Ray& r, float& cut, ctr_t& nn,
                                          bool sort, LeafFn&& leaf) {
    constexpr int CAP = ANY ? kAnyStack : kBvhStack;
    uint2* stk = g_bstk + threadIdx.x;
    unsigned* stw = g_astk + threadIdx.x;
    int sp = 0;
    bool overflow = false;
    int lf = 0, lc = 0;
    // Speculative while-while (Aila & Laine 2009): a lane that holds a leaf keeps opening nodes while other lanes
    // of its wave are still looking for theirs, so the node steps the wave executes anyway do useful work (CFG3:
    // 29 % of the lanes of a node step were busy without it).  node: an internal node to open (>= 0), none (-1), or
    // a second leaf's word (< -1) waiting until the held leaf (lf, lc) is tested.  A held leaf's triangles are
    // tested after those nodes, with the cut of that time: more nodes may be opened, the answer is the same (the
    // canonical rule does not depend on the order; a stack overflow still makes the ray ambiguous).
    int node = 0;
    while (true) {
        while (true) {
            const bool more = node >= 0 || (node == -1 && sp > 0);
            if (__ballot(lc == 0 && more) == 0) break;  // every lane holds a leaf or is done
            if (!more) continue;
            // pop, then open a popped internal node in the same step (the lanes popping and the lanes holding a
            // node open theirs together instead of in alternating steps)
            if (node == -1) {
                if constexpr (ANY) {
                    --sp;
                    node = (int)stw[sp * kBlock];
                } else {
                    while (sp > 0) {
                        const uint2 e = stk[--sp * kBlock];
                        if (__uint_as_float(e.y & 0x7ffffff8u) <= cut) {  // (entered beyond the current cut: dropped)
                            node = (int)e.x;
                            break;
                        }
                    }
                }
            }
            if (node >= 0) {
                RT_SIMD_TICK(ANY ? 4 : 0);
                const BvhNode8 bn = load_node8(nodes, node);
                nn += __popc(bn.N1.w);
                unsigned k[8];
                node_keys(bn, r, cut, k, sort);
                node = -1;
#pragma unroll
                for (int i = 7; i >= 1; --i)
                    if (k[i] != kNoChild) {
                        if (sp >= CAP) overflow = true;
                        else if constexpr (ANY) stw[sp++ * kBlock] = (unsigned)child_word(bn, k[i]);
                        else stk[sp++ * kBlock] = make_uint2((unsigned)child_word(bn, k[i]), k[i]);
                    }
                if (k[0] != kNoChild) node = child_word(bn, k[0]);
            }
            if (node < -1 && lc == 0) {
                decode_leaf(node, lf, lc);
                node = -1;
            }
        }
        if (lc == 0) break;  // nothing held, nothing left: this lane's walk is over
        // at most kLeafStep triangles per leaf phase (the rest stays held)
        const int m = lc < kLeafStep ? lc : kLeafStep;
        const bool done = leaf(lf, m);
        lf += m;
        lc -= m;
        if (done) break;
        if (lc == 0 && node < -1) {
            decode_leaf(node, lf, lc);
            node = -1;
        }
    }
    return !overflow;
}

// closest hit over the BVH: returns the triangle id (or -1) with (b0, b1, b2, t); amb = the BFS must decide
template <int KZ>
__device__ __forceinline__ int bvh_closest(const DevScene& sc, int set, V3 o, V3 d, float tMaxInit, float& rb0,
                                           float& rb1, float& rb2, float& rt, ctr_t& nn, ctr_t& nt, bool& amb) {
    if (bvh_refuses(sc, o, d)) {
        amb = true;
        return -1;
    }
    const float* __restrict__ tiles = sc.btiles[set];
    Bvh8Ray r;
    r.inv = bvh_inv(d);
    r.oi = v3(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
    const TriRay R = make_triray<KZ>(o, d);
    float cut = tMaxInit, t2 = __builtin_inff();
    int best = -1, second = -1;  // tile indices (the winner's triangle id is read once, after the walk)
    const bool ok = bvh8_walk<false>(sc.bvh[set], r, cut, nn, true, [&](int lf, int lc) {
        // the next triangle's tile is loaded while this one is tested (a leaf's tiles are contiguous)
        const float* tp = tiles + 9 * lf;
        float4 A = ld_f4u(tp), B = ld_f4u(tp + 4);
        float C = tp[8];
        for (int k = 0; k < lc; ++k) {
            float4 nA = A, nB = B;
            float nC = C;
            if (k + 1 < lc) { nA = ld_f4u(tp + 9 * k + 9); nB = ld_f4u(tp + 9 * k + 13); nC = tp[9 * k + 17]; }
            ++nt;
            RT_SIMD_TICK(2);
            float b0, b1, b2, t;
            if (tri_intersect<KZ>(R, cut, A, B, make_float4(C, 0.f, 0.f, 0.f), b0, b1, b2, t) && t < cut) {
                if (best < 0 || t < rt) {
                    t2 = best < 0 ? t2 : rt;
                    second = best;
                    best = lf + k;
                    rb0 = b0; rb1 = b1; rb2 = b2; rt = t;
                    const float c2 = t + 2.f * canon_window(t, sc.wabs);
                    cut = c2 < cut ? c2 : cut;
                } else if (t < t2) {
                    second = lf + k;
                    t2 = t;
                }
            }
            A = nA; B = nB; C = nC;
        }
        return false;
    });
    amb = !ok || (second >= 0 && t2 <= rt + canon_window(rt, sc.wabs));
    return best >= 0 ? sc.btid[set][best] : -1;
}

// any hit over the BVH with a fixed tMax: 0 = occluded, -1 = not; amb = only window hits were found.  The children are
// pushed in slot order, unsorted: any order gives the same answer, and the sorting network cost more than the
// nearer-first order saved (r05_ab24: CFG3 +0.8 %).  RT_ANY_SORT=1 (variant builds): nearest-first.
#ifndef RT_ANY_SORT
#define RT_ANY_SORT 0
#endif
template <int KZ>
__device__ __forceinline__ int bvh_anyhit(const DevScene& sc, int set, V3 o, V3 d, float tMax, ctr_t& nn, ctr_t& nt,
                                          bool& amb) {
    if (bvh_refuses(sc, o, d)) {
        amb = true;
        return -1;
    }
    const float* __restrict__ tiles = sc.btiles[kBvhAny];  // (shadow rays: every triangle, set 0)
    Bvh8Ray r;
    r.inv = bvh_inv(d);
    r.oi = v3(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
    const TriRay R = make_triray<KZ>(o, d);
    const float sure = tMax - canon_window(tMax, sc.wabs);
    bool window = false, occluded = false;
    float cut = tMax;
    const bool ok = bvh8_walk<true>(sc.bvh[kBvhAny], r, cut, nn, RT_ANY_SORT != 0, [&](int lf, int lc) {
        const float* tp = tiles + 9 * lf;
        float4 A = ld_f4u(tp), B = ld_f4u(tp + 4);
        float C = tp[8];
        for (int k = 0; k < lc; ++k) {
            float4 nA = A, nB = B;
            float nC = C;
            if (k + 1 < lc) { nA = ld_f4u(tp + 9 * k + 9); nB = ld_f4u(tp + 9 * k + 13); nC = tp[9 * k + 17]; }
            ++nt;
            RT_SIMD_TICK(6);
            float b0, b1, b2, t;
            if (tri_intersect<KZ>(R, tMax, A, B, make_float4(C, 0.f, 0.f, 0.f), b0, b1, b2, t) && t < tMax) {
                if (t < sure) { occluded = true; return true; }
                window = true;
            }
            A = nA; B = nB; C = nC;
        }
        return false;
    });
    if (occluded) { amb = false; return 0; }
    amb = window || !ok;
    return -1;
}

template <int QCAP, bool ANYHIT, int KZ, bool DFS>
__device__ __forceinline__ int traverse_kz(const DevScene& sc, int set, V3 o, V3 d, float tMax, float& b0, float& b1,
                                           float& b2, float& t, ctr_t& nn, ctr_t& nt, ctr_t& nfb) {
    if constexpr (QCAP != 1) {
        bool amb = false;
        const int r = ANYHIT ? bvh_anyhit<KZ>(sc, set, o, d, tMax, nn, nt, amb)
                             : bvh_closest<KZ>(sc, set, o, d, tMax, b0, b1, b2, t, nn, nt, amb);
        if (!amb) return r;
        ++nfb;  // ambiguous (rare): the reference BFS decides, with the wave's other lanes done with the BVH
    }
    return traverse<QCAP, ANYHIT, KZ, DFS>(sc, set, o, d, tMax, b0, b1, b2, t, nn, nt);
}

// When every active lane of the wave has the same dominant ray axis (camera rays) the watertight test's coordinate
// permutation is resolved at compile time; otherwise per lane.
template <int QCAP, bool ANYHIT, bool DFS = false>
__device__ __forceinline__ int traverse_any(const DevScene& sc, int set, V3 o, V3 d, float tMax, float& b0, float& b1,
                                            float& b2, float& t, ctr_t& nn, ctr_t& nt, ctr_t& nfb) {
    int kz = dominant_axis(d);
    uint64_t act = __ballot(true);
    if (__ballot(kz == 2) == act) return traverse_kz<QCAP, ANYHIT, 2, DFS>(sc, set, o, d, tMax, b0, b1, b2, t, nn, nt, nfb);
    if (__ballot(kz == 0) == act) return traverse_kz<QCAP, ANYHIT, 0, DFS>(sc, set, o, d, tMax, b0, b1, b2, t, nn, nt, nfb);
    if (__ballot(kz == 1) == act) return traverse_kz<QCAP, ANYHIT, 1, DFS>(sc, set, o, d, tMax, b0, b1, b2, t, nn, nt, nfb);
    return traverse_kz<QCAP, ANYHIT, -1, DFS>(sc, set, o, d, tMax, b0, b1, b2, t, nn, nt, nfb);
}

// Multi-level scenes: the BVH walk alone (no reference-BFS fallback in the calling kernel, whose register budget it
// would set: trace 128 VGPRs + spill with it, 106 without); amb = the canonical rule could not decide, and the caller
// hands the ray (or its path vertex) to a kernel that runs the exact traversal.
// KZSPEC: waves whose rays share a dominant axis take a copy of the walk with the watertight test's permutation
// resolved at compile time (4 copies of the walk); otherwise one copy with the permutation per lane.
template <bool ANYHIT, bool KZSPEC = true>
__device__ __forceinline__ int traverse_bvh(const DevScene& sc, int set, V3 o, V3 d, float tMax, float& b0, float& b1,
                                            float& b2, float& t, ctr_t& nn, ctr_t& nt, bool& amb) {
    int kz = dominant_axis(d);
    uint64_t act = __ballot(true);
#define RT_BVH_KZ(K) \
    return ANYHIT ? bvh_anyhit<K>(sc, set, o, d, tMax, nn, nt, amb) : bvh_closest<K>(sc, set, o, d, tMax, b0, b1, b2, t, nn, nt, amb)
    if constexpr (!KZSPEC) RT_BVH_KZ(-1);
    if (__ballot(kz == 2) == act) RT_BVH_KZ(2);
    if (__ballot(kz == 0) == act) RT_BVH_KZ(0);
    if (__ballot(kz == 1) == act) RT_BVH_KZ(1);
    RT_BVH_KZ(-1);
#undef RT_BVH_KZ
}

// Register budgets (amdgpu_waves_per_eu) of the multi-level instantiations: 4 waves/SIMD (128 VGPRs) on the trace,
// path shade and mixed-scene shade kernels (CFG3 121 -> 144, CFG4 87 -> 111 Msamples/s; 5 waves spill too much).
// The single-leaf instantiations (107 / 123 VGPRs) are unbudgeted (5 waves: trace -2 %, shade -7 %).
// These budgets (RT_*_WAVES), the any-hit stack depth (RT_ANY_STACK), the radix digit widths (rt_sort.hip) and the
// staged BVH levels (rt_internal.h) are numeric tuning constants a variant build may override (Makefile
// `variants`); RT_SIMD_STATS selects the SIMD-efficiency measurement build.  No code path is switched by a macro.
#ifndef RT_MULTI_WAVES
#define RT_MULTI_WAVES 4
#endif
#ifndef RT_TRACE_WAVES
#define RT_TRACE_WAVES RT_MULTI_WAVES  // the multi-level closest-hit trace (variant builds)
#endif
#ifndef RT_TRACE1_WAVES
#define RT_TRACE1_WAVES 1  // the single-leaf closest-hit trace: unbudgeted (variant builds)
#endif
#define RT_WAVES_ATTR(Q) __attribute__((amdgpu_waves_per_eu((Q) == 1 ? RT_TRACE1_WAVES : RT_TRACE_WAVES)))
#ifndef RT_SHADE1_WAVES
#define RT_SHADE1_WAVES 4  // the single-leaf simple-path shade (Cornell)
#endif
#ifndef RT_SHADE_WAVES
#define RT_SHADE_WAVES RT_MULTI_WAVES  // the simple-path shade (its shadow rays' any-hit walks)
#endif

// The analytic shapes after the octree's closest hit, with the running tMax (hitB = the object-space
// point for a shape), then the hit record at queue position p.
template <bool CULL>
__device__ __forceinline__ int finish_closest(const DevScene& sc, const TraceIO& io, int p, float4 o4, float4 d4,
                                              int prim, float b0, float b1, float b2, float t) {
    if (sc.n_shapes) {
        float tm = prim >= 0 ? t : 3.402823466e+38f;
        for (int si = 0; si < sc.n_shapes; ++si) {
            DevShape sh = ldconst(sc.shapes, si);
            V3 ph;
            float th;
            if (shape_isect<CULL>(sh, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z), tm, ph, th)) {
                prim = sc.n_tris + si; b0 = ph.x; b1 = ph.y; b2 = ph.z; t = th; tm = th;
            }
        }
    }
    io.hitB[p] = make_float4(b0, b1, b2, t);
    io.hitPrim[p] = prim;
    return prim;
}

// Multi-level closest-hit walks with the watertight test's permutation specialised per wave (RT_TRACE_KZ=1) or per
// lane (0; one copy of the walk instead of four).
#ifndef RT_TRACE_KZ
#define RT_TRACE_KZ 1
#endif

// FBL (multi-level scenes, path mode: io.fb_pos): the BVH walk alone, the ambiguous rays listed for k_trace_fallback;
// otherwise the reference BFS runs inline for them.
template <int QCAP, bool FBL>
__global__ void __launch_bounds__(kBlock) RT_WAVES_ATTR(QCAP) k_trace_closest(DevScene sc, TraceIO io, unsigned long long* ctr) {
    stage_scene<QCAP, false>(sc, io.set);
    if (io.zero && blockIdx.x == 0)
        for (int i = threadIdx.x; i < kQRegion; i += blockDim.x) io.zero[i] = 0;
    ctr_t nn = 0, nt = 0, nh = 0, nr = 0, nfb = 0, novf = 0;
    // one ray at queue position p: octree (BVH / BFS), then the analytic shapes
    auto trace_one = [&](int p, float4 o4, float4 d4) __attribute__((always_inline)) {
        float b0 = 0, b1 = 0, b2 = 0, t = 0;
        int prim;
        if constexpr (QCAP != 1 && FBL) {
            bool amb = false;
            prim = traverse_bvh<false, RT_TRACE_KZ != 0>(sc, io.set, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z),
                                                         3.402823466e+38f, b0, b1, b2, t, nn, nt, amb);
            if (amb) {  // (multi-level scenes run on tickets, below: this static-chunk form is not launched)
                ++nfb;
                io.fb_pos[atomicAdd(io.fb_len, 1)] = p;
                return;
            }
        } else {
            prim = traverse_any<QCAP, false>(sc, io.set, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z), 3.402823466e+38f,
                                             b0, b1, b2, t, nn, nt, nfb);
        }
        prim = finish_closest<QCAP != 1>(sc, io, p, o4, d4, prim, b0, b1, b2, t);
        nh += prim >= 0;
        nr += 1;
    };
    // no block-level synchronisation here.  Static chunks (single leaf, dense queues) or per-wave tickets.  One shard
    // (single leaf): a thread's items are k(i) = (block + (i / S) grid) S kBlock + (i % S) kBlock + thread,
    // S = kStaticItems, and the next item's ray is loaded while the current one is traced.
    if (!io.ticket && io.q.ns == 1) {
        const int n = q_len(io.q, 0);
        auto item = [&](int i) {
            return (blockIdx.x + (i / kStaticItems) * gridDim.x) * kChunk + (i % kStaticItems) * kBlock +
                   (int)threadIdx.x;
        };
        int k = item(0);
        float4 o4 = make_float4(0, 0, 0, 0), d4 = o4;
        if (k < n) { o4 = io.rayO[k << io.rsh]; d4 = io.rayD[k << io.rsh]; }
        for (int i = 1; k < n; ++i) {
            const int kn = item(i);
            float4 on = o4, dn = d4;
            if (kn < n) { on = io.rayO[kn << io.rsh]; dn = io.rayD[kn << io.rsh]; }
            trace_one(k, o4, d4);
            k = kn; o4 = on; d4 = dn;
        }
    } else if (!io.ticket) {
        StaticChunks ch(io.q);
        int base;
        while (ch.next(base)) {
#pragma unroll 1
            for (int r = 0; r < kStaticItems; ++r) {  // (one copy of the traversal: no unrolling)
                const int idx = base + r * kBlock + (int)threadIdx.x;
                if (idx < ch.len) {
                    const int p = ch.j * io.q.S + idx;
                    trace_one(p, io.rayO[p << io.rsh], io.rayD[p << io.rsh]);
                }
            }
        }
    } else {
        // Multi-level scenes, sorted bounces: position p's ray is the queue's ray perm[p] (rt_sort.hip), gathered
        // here into the sorted side queue `so` (coalesced stores) on its way to the traversal
        WaveTickets tk(io.ticket, io.q);
        int j, base;
        while (tk.next(j, base)) {
            const int idx = base + lane_id();
            if constexpr (FBL && QCAP != 1) {
                // the BVH walk per lane; then the wave resolves its ambiguous rays one after the other with the
                // wave-cooperative BFS (all lanes active), so no lane holds the per-thread BFS's registers
                const bool live = idx < tk.len;
                const int p = j * io.q.S + idx;
                float4 o4 = make_float4(0, 0, 0, 0), d4 = o4;
                float b0 = 0, b1 = 0, b2 = 0, t = 0;
                int prim = -1;
                bool amb = false;
                if (live) {
                    const int src = io.perm ? io.perm[p] : p;
                    o4 = io.rayO[src << io.rsh];
                    d4 = io.rayD[src << io.rsh];
                    if (io.so) { io.so[2 * p] = o4; io.so[2 * p + 1] = d4; }
                    prim = traverse_bvh<false, RT_TRACE_KZ != 0>(sc, io.set, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z),
                                                                 3.402823466e+38f, b0, b1, b2, t, nn, nt, amb);
                }
                // (coop_ok == 0: the octree's BFS queue may exceed the FIFO, and the host launches k_trace_fallback:
                // the ambiguous rays are listed for it directly)
                uint64_t am = sc.coop_ok ? __ballot(live && amb) : 0ull;
                while (am) {
                    const int L = __builtin_ctzll(am);
                    am &= am - 1;
                    const V3 oL = v3(__shfl(o4.x, L), __shfl(o4.y, L), __shfl(o4.z, L));
                    const V3 dL = v3(__shfl(d4.x, L), __shfl(d4.y, L), __shfl(d4.z, L));
                    int cp = -1;
                    float c0 = 0.f, c1 = 0.f, c2 = 0.f, ctt = 0.f;  // (a miss stores zeros, as the BFS does)
                    ctr_t cnn = 0, cnt = 0;
                    const bool ok = bfs_coop<false>(sc, io.set, oL, dL, 3.402823466e+38f, coop_fifo_bstk(), cp, c0, c1,
                                                    c2, ctt, cnn, cnt);
                    if (lane_id() == L) {
                        ++nfb;
                        nn += cnn;
                        nt += cnt;
                        if (ok) { prim = cp; b0 = c0; b1 = c1; b2 = c2; t = ctt; amb = false; }
                        else ++novf;
                    }
                }
                if (live) {
                    if (amb) {  // (coop_ok == 0: k_trace_fallback's per-thread BFS decides the ray)
                        io.fb_pos[atomicAdd(io.fb_len, 1)] = p;
                        if (!sc.coop_ok) ++nfb;  // (coop rays are counted above)
                        // coop_ok promised that the FIFO cannot overflow, so no fallback launch follows: a broken
                        // promise is counted (C_COOPOVF, rt_stats coop_overflows; the tests require 0) and the ray
                        // stored as a miss instead of leaving the previous bounce's hit at this position
                        else { io.hitPrim[p] = -1; io.hitB[p] = make_float4(0.f, 0.f, 0.f, 0.f); }
                    } else {
                        prim = finish_closest<QCAP != 1>(sc, io, p, o4, d4, prim, b0, b1, b2, t);
                        nh += prim >= 0;
                        nr += 1;
                    }
                }
            } else if (idx < tk.len) {
                const int p = j * io.q.S + idx;
                const int src = io.perm ? io.perm[p] : p;
                const float4 o4 = io.rayO[src << io.rsh], d4 = io.rayD[src << io.rsh];
                if (io.so) { io.so[2 * p] = o4; io.so[2 * p + 1] = d4; }
                trace_one(p, o4, d4);
            }
        }
    }
    count_add(ctr, C_NODES, nn);
    count_add(ctr, C_TRIS, nt);
    count_add(ctr, C_HITS, nh);
    count_add(ctr, C_RAYS, nr);
    count_add(ctr, C_FALLBACK, nfb);
    if constexpr (QCAP != 1) count_add(ctr, C_COOPOVF, novf);
    if constexpr (QCAP != 1) simd_flush();
}

// The rays k_trace_closest<Q, true> listed (io.fb_pos): the reference BFS (Octtree_Model.h:66-127, exact order and
// ties) then the shapes, on a small grid right after it.  Their rays are read where the trace kernel read them: the
// sorted side queue it wrote (io.so) or the queue itself.
template <int QCAP>
__global__ void __launch_bounds__(kBlock) k_trace_fallback(DevScene sc, TraceIO io, unsigned long long* ctr) {
    ctr_t nn = 0, nt = 0, nh = 0, nr = 0;
    const int n = *io.fb_len;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const int p = io.fb_pos[k];
        const float4 o4 = io.so ? io.so[2 * p] : io.rayO[p << io.rsh];
        const float4 d4 = io.so ? io.so[2 * p + 1] : io.rayD[p << io.rsh];
        float b0 = 0, b1 = 0, b2 = 0, t = 0;
        int prim = traverse<QCAP, false, -1>(sc, io.set, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z), 3.402823466e+38f,
                                             b0, b1, b2, t, nn, nt);
        prim = finish_closest<QCAP != 1>(sc, io, p, o4, d4, prim, b0, b1, b2, t);
        nh += prim >= 0;
        nr += 1;
    }
    count_add(ctr, C_NODES, nn);
    count_add(ctr, C_TRIS, nt);
    count_add(ctr, C_HITS, nh);
    count_add(ctr, C_RAYS, nr);
}

// Material bins of a mixed multi-level scene's bounce (BinIO): every hit's queue position is appended to the index
// list of its material class, shard by shard, in queue order within a chunk; misses go to no bin (no miss work; at
// lean depth 0 their L = 0 is stored here).  A pass over the hit ids of its own (in the trace kernel the appends cost
// registers the traversal needs).  A block takes chunks of kBinItems x 256 consecutive positions of one shard: it
// counts each class (wave ballots, LDS), makes ONE atomic per class and chunk (per-wave appends on the per-shard
// class counters saturated them: 313 us per launch), then writes the positions at their ranks.
static constexpr int kBinItems = 8;
__global__ void __launch_bounds__(kBlock) k_bin_materials(DevScene sc, BinIO io) {
    constexpr int NW = kBlock / 64, CH = kBinItems * kBlock;
    __shared__ int wc[kMatClasses][kBinItems][NW];  // per (class, item round, wave): count, then exclusive start
    __shared__ int base[kMatClasses];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const bool lds_mats = stage_materials(sc);
    int mx = 0;
#pragma unroll
    for (int j = 0; j < kShards; ++j) {
        const int l = j < io.q.ns ? q_len(io.q, j) : 0;
        mx = l > mx ? l : mx;
    }
    const int per_shard = (mx + CH - 1) / CH, nent = io.q.ns * per_shard;
    for (int e = blockIdx.x; e < nent; e += gridDim.x) {  // entry e = chunk e / ns of shard e % ns
        const int j = e % io.q.ns, c0 = (e / io.q.ns) * CH, len = q_len(io.q, j);
        if (c0 >= len) continue;  // (block-uniform)
        int cls[kBinItems];
#pragma unroll
        for (int r = 0; r < kBinItems; ++r) {
            const int idx = c0 + r * kBlock + (int)threadIdx.x;
            cls[r] = -1;
            if (idx < len) {
                const int prim = io.hitPrim[j * io.q.S + idx];
                if (prim >= 0)
                    cls[r] = mat_at(sc, lds_mats, prim < sc.n_tris ? sc.triMaterial[prim] : sc.shapes[prim - sc.n_tris].material).cls;
                else if (io.rayO) {  // lean depth 0: a camera ray that missed ends with L = 0
                    const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                    rstore8(io.rec, __float_as_int(io.rayO[2 * (j * io.q.S + idx)].w), R_L, z);
                }
            }
        }
#pragma unroll
        for (int c = 0; c < kMatClasses; ++c)
#pragma unroll
            for (int r = 0; r < kBinItems; ++r) {
                const uint64_t m = __ballot(cls[r] == c);
                if (lane == 0) wc[c][r][w] = __popcll(m);
            }
        __syncthreads();
        if (threadIdx.x < kMatClasses) {  // exclusive starts in (round, wave) order, then the chunk's one atomic
            const int c = threadIdx.x;
            int t = 0;
            for (int r = 0; r < kBinItems; ++r)
                for (int i = 0; i < NW; ++i) { const int v = wc[c][r][i]; wc[c][r][i] = t; t += v; }
            base[c] = t ? atomicAdd(io.len + (c * kShards + j) * kQStride, t) : 0;
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < kMatClasses; ++c)
#pragma unroll
            for (int r = 0; r < kBinItems; ++r) {
                const uint64_t m = __ballot(cls[r] == c);
                if (cls[r] == c)
                    io.idx[c][j * io.q.S + base[c] + wc[c][r][w] + __popcll(m & lt)] = j * io.q.S + c0 + r * kBlock + (int)threadIdx.x;
            }
        __syncthreads();  // (wc / base are rewritten by the block's next chunk)
    }
}

// The last depth's emitter filter (EmitIO, rt_internal.h): a ray is kept when some emissive triangle passes the
// watertight test (Shapes.h:1101-1260) or some emissive shape its intersection test, each with tMax = FLT_MAX.  The
// closest-hit traversal can only return an emitter whose own test passed with a smaller tMax, and both tests are
// monotone in tMax, so a dropped ray's closest hit is never an emitter: the shade kernel would have added nothing.
__global__ void __launch_bounds__(kBlock) k_emitter_filter(DevScene sc, EmitIO io) {
    __shared__ int lds[kBlock / 64 + 1];
    QueueItems<false> items(nullptr, io.q);
    int qj, qidx;
    bool live;
    while (items.next(qj, qidx, live)) {
        const int k = qj * io.q.S + qidx;
        float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = o4;
        bool keep = false;
        if (live) {
            o4 = io.rayO[2 * k];
            d4 = io.rayO[2 * k + 1];
            const V3 o = v3(o4.x, o4.y, o4.z), d = v3(d4.x, d4.y, d4.z);
            const TriRay R = make_triray<-1>(o, d);
            for (int e = 0; e < sc.n_emit_tris && !keep; ++e) {
                const int t = sc.emit_tris[e];
                const float4 P0 = sc.triWorld[3 * t], P1 = sc.triWorld[3 * t + 1], P2 = sc.triWorld[3 * t + 2];
                float b0, b1, b2, tt;
                keep = tri_intersect<-1>(R, 3.402823466e+38f, make_float4(P0.x, P0.y, P0.z, P1.x),
                                         make_float4(P1.y, P1.z, P2.x, P2.y), make_float4(P2.z, 0.f, 0.f, 0.f), b0, b1,
                                         b2, tt);
            }
            for (int e = 0; e < sc.n_emit_shapes && !keep; ++e) {
                const DevShape sh = ldconst(sc.shapes, sc.emit_shapes[e]);
                V3 ph;
                float th;
                keep = shape_isect(sh, o, d, 3.402823466e+38f, ph, th);
            }
        }
        const int p = block_append(io.nCount + qj * kQStride, keep, lds) + qj * io.q.S;
        if (keep) {
            io.nO[2 * p] = o4;
            io.nO[2 * p + 1] = d4;
        }
    }
}

// ======================================================================= K3 reference shading + film
// RayTracerTestApp.h:218-284 (Li, active branch):  0.3·F1(λ) + clamp(n·(0,0,-1), 0, 1)·(D65(λ)·albedo(λ)),
// n = object-space interpolated normal flipped against the ray (Shapes.h:1066-1075).
__device__ __forceinline__ void li_reference(const DevScene& sc, const DevSpectra* sp, const ShadeRefIO& io, int s,
                                             const float lam[8], float L[8]) {
    int prim = io.hitPrim[s];
#pragma unroll
    for (int i = 0; i < 8; ++i) L[i] = 0.f;
    if (prim < 0) return;
    float4 bb = io.hitB[s];
    float4 n1 = sc.triNormal[3 * prim], n2 = sc.triNormal[3 * prim + 1], n3 = sc.triNormal[3 * prim + 2];
    V3 n = vnorm(vadd(vadd(vmul(v3(n1.x, n1.y, n1.z), bb.x), vmul(v3(n2.x, n2.y, n2.z), bb.y)),
                      vmul(v3(n3.x, n3.y, n3.z), bb.z)));
    float4 d4 = io.rayD[s << io.rsh];
    V3 rd = vnorm(v3(d4.x, d4.y, d4.z));  // TriangleIntersect::rayd (Shapes.h:1259)
    if (vdot(n, rd) > 0) n = v3(-n.x, -n.y, -n.z);
    float cosv = gclamp(vdot(n, v3(0, 0, -1)), 0.0f, 1.0f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float light = (io.illum_scale * sigmoid_eval(0, 0, io.illum_c2, lam[i])) * d65_query(sp, lam[i]);
        float amb = piecewise_query(sp->f1_lambda, sp->f1_value, sp->f1_n, lam[i]) * 0.3f;
        float mat = sigmoid_eval(0, 0, io.albedo_c2, lam[i]);
        float r = 0.0f + amb;
        r += (light * mat) * cosv;
        L[i] = r;
    }
}

// Film accumulation (RayTracerTestApp.h:330-337): each thread owns one pixel and adds the batch's sample
// indices in increasing order — the same per-pixel summation order as the reference's passes.
__global__ void __launch_bounds__(kBlock) k_ref_shade_film(DevScene sc, const DevSpectra* sp, DevFilm film,
                                                           ShadeRefIO io, unsigned long long* ctr) {
    stage_spectra(sp);
    ctr_t ns = 0;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < io.n_pixels; j += gridDim.x * blockDim.x) {
        int pixel = io.work_pixels[j];
        float4 f = io.film[pixel];
        for (int i = 0; i < io.n_index; ++i) {
            int s = i * io.n_pixels + j;
            float lam[8], pdf[8], L[8], rgb[3];
            load8(io.lamA, io.lamB, s, lam);
            load8(io.pdfA, io.pdfB, s, pdf);
            li_reference(sc, sp, io, s, lam, L);
            to_sensor_rgb_spk(sp, L, lam, pdf, film.imaging_ratio, rgb);
            const float w = 1.0f;  // FilterSample::weight (Box and Triangle both return 1)
            f.x += w * gclamp(rgb[0], 0.0f, 1.0f);
            f.y += w * gclamp(rgb[1], 0.0f, 1.0f);
            f.z += w * gclamp(rgb[2], 0.0f, 1.0f);
            f.w += w;
            ++ns;
        }
        io.film[pixel] = f;
    }
    count_add(ctr, C_SAMPLES, ns);
}

__global__ void k_records(DevScene sc, const DevSpectra* sp, DevFilm film, ShadeRefIO sio, RecordIO io) {
    stage_spectra(sp);
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= io.n) return;
    float lam[8], pdf[8], L[8], rgb[3];
    load8(io.lamA, io.lamB, s, lam);
    load8(io.pdfA, io.pdfB, s, pdf);
    li_reference(sc, sp, sio, s, lam, L);
    to_sensor_rgb_spk(sp, L, lam, pdf, film.imaging_ratio, rgb);
    float* r = io.out + (size_t)s * io.stride;
    for (int i = 0; i < 8; ++i) { r[i] = lam[i]; r[8 + i] = pdf[i]; }
    float4 o = io.rayO[s << io.rsh], d = io.rayD[s << io.rsh];
    r[16] = o.x; r[17] = o.y; r[18] = o.z; r[19] = d.x; r[20] = d.y; r[21] = d.z;
    int prim = io.hitPrim[s];
    ((int*)r)[22] = prim;
    float4 hb = prim < 0 ? make_float4(0, 0, 0, 0) : io.hitB[s];
    r[23] = hb.x; r[24] = hb.y; r[25] = hb.z; r[26] = hb.w;
    for (int i = 0; i < 8; ++i) r[27 + i] = L[i];
    for (int c = 0; c < 3; ++c) r[35 + c] = gclamp(rgb[c], 0.0f, 1.0f);
    r[38] = 1.0f;
}

// ============================================================================ path mode (build-defined)
// One bounce of the diffuse path integrator (pbrt-v4 SimplePathIntegrator semantics): emitter hit →
// Le at depth 0 only (one-sided), then terminate; otherwise NEE on the quad light (Get2D, shadow ray traced inline,
// pending contribution added on a miss) and a cosine-hemisphere bounce (Get2D, β *= R) appended to the next queue.
// Sampler state (PCG state + dimension) lives per path slot.
// dim_loaded / pixel_loaded >= 0: the dimension / pixel id from an R_MISC the caller already read (mixed scenes:
// k_generate keeps the pixel in R_MISC.w), so the slot's pixel is not gathered from the work list
__device__ __forceinline__ void restore_sampler(const SampleIds& ids, const DevFilm& film, const PathIO& io, int slot,
                                                Smp& sm, int smp_kind, int smp_seed, int dim_loaded = -1,
                                                int pixel_loaded = -1) {
    // the PCG state; the increment SetSequence gave the path (rng.h:36-39) is recomputed from the pixel hash instead
    // of read back (Sobol keeps its index in the state).  The record layout keeps the pixel id beside the state
    // (k_generate), so one 16-B load gives both and the work list is not gathered.
    uint2 st;
    if (io.rec.rng8) {
        st = rng8_state(io.rec)[slot];
    } else {
        const uint4 rs = *reinterpret_cast<const uint4*>(recf(io.rec, slot, R_RNG));
        st = make_uint2(rs.x, rs.y);
        pixel_loaded = (int)rs.z;
    }
    int pixel, index, x, y;
    if (pixel_loaded >= 0 && !ids.ex_pixel) {
        pixel = pixel_loaded;
        index = ids.index_begin + (ids.np_div.m ? intdiv(slot, ids.np_div) : slot / ids.n_pixels);
    } else {
        sample_of(ids, slot, pixel, index);
    }
    pixel_xy(film, pixel, x, y);
    sm.rng.state = (uint64_t)st.x | ((uint64_t)st.y << 32);
    sm.rng.inc = smp_kind == 2 ? 0ull : (hash_pixel(x, y, smp_seed) << 1u) | 1u;
    sm.px = x; sm.py = y; sm.index = index;
    sm.dim = io.dim >= 0 ? io.dim : dim_loaded >= 0 ? dim_loaded : __float_as_int(recf(io.rec, slot, R_MISC)->x);
}
// the PCG increment of a path never changes after generation: only the 8-byte state half is written back
// store_dim = false: the caller writes the dimension with the rest of R_MISC (one 16-B store)
__device__ __forceinline__ void save_sampler(const PathIO& io, int slot, const Smp& sm, bool store_dim = true) {
    const uint2 st = make_uint2((uint32_t)sm.rng.state, (uint32_t)(sm.rng.state >> 32));
    if (io.rec.rng8) rng8_state(io.rec)[slot] = st;
    else *reinterpret_cast<uint2*>(recf(io.rec, slot, R_RNG)) = st;
    if (io.dim < 0 && store_dim) *reinterpret_cast<int*>(recf(io.rec, slot, R_MISC)) = sm.dim;
}
// cosine-hemisphere direction (Sampling.h:449-454) in the pbrt CoordinateSystem frame of nrm; false when z == 0
__device__ __forceinline__ bool cosine_bounce(float u0, float u1, V3 nrm, V3& wi, float& z) {
    float dx, dy;
    disk_concentric(u0, u1, dx, dy);
    z = 1 - dx * dx - dy * dy;
    z = sqrtf(z > 0.f ? z : 0.f);  // SafeSqrt: std::max(0.f, x)
    if (z == 0) return false;
    float sign = copysignf(1.0f, nrm.z);
    float a = -1 / (sign + nrm.z);
    float b = nrm.x * nrm.y * a;
    V3 ss = v3(1 + sign * (nrm.x * nrm.x) * a, sign * b, -sign * nrm.x);
    V3 tt = v3(b, sign + (nrm.y * nrm.y) * a, -nrm.y);
    wi = vadd(vadd(vmul(ss, dx), vmul(tt, dy)), vmul(nrm, z));
    return true;
}

template <int QCAP>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(QCAP == 1 ? RT_SHADE1_WAVES : RT_SHADE_WAVES))) k_path_shade(DevScene sc, const DevSpectra* sp, DevSampler smp,
                                                                         DevFilm film, SampleIds ids, PathIO io,
                                                                         unsigned long long* ctr, ShadowQueueIO shq) {
    const float InvPi = 0.31830988618379067154f;
    bool lds_tris = false;
    stage_spectra(sp);
    stage_scene<QCAP>(sc, 0);
    if constexpr (QCAP == 1) lds_tris = stage_tris1(sc);
    __shared__ int lds[2 * (kBlock / 64) + 1];
    // single leaf: the first item of a static chunk parks its bounce ray here; the second item appends both (one
    // atomic and one round of barriers per chunk: Cornell +3.5 %, r03)
    __shared__ float4 pend[QCAP == 1 ? 2 * kBlock : 1];
    bool pend0 = false;
    ctr_t snn = 0, snt = 0, nsh = 0, sfb = 0, novf = 0;
    // lean depth 0: k_generate stored no β = 1 / L = 0, so they start in registers and every path's L is written
    const bool d0 = io.lean && io.depth == 0;
    // multi-level octrees: per-wave tickets and appends (per-ray cost varies by 100x); single leaf: per block
    constexpr bool WAVE = QCAP != 1;
    // single leaf: the host gives the queues one shard (rt_host.cpp nsh)
    std::conditional_t<QCAP == 1, QueueItemsOne, QueueItems<WAVE>> items(io.ticket, io.q);
    int qj, qidx;
    bool live;
    while (items.next(qj, qidx, live)) {
        const int k = qj * io.q.S + qidx;  // queue position
        bool wantShadow = false, wantNext = false, storedL = false;
        float4 nO = make_float4(0, 0, 0, 0), nD = nO;
        V3 so = v3(0, 0, 0), sd = so;
        float stmax = 0.f;
        float Ld[8];
        int slot = -1;
        if (live) {
            // (the ray's origin carries its slot; at depth 0 the queue is k_generate's dense camera queue, slot = k,
            // so the slot's state loads need not wait for the ray's)
            slot = io.depth == 0 ? k : __float_as_int(io.rayO[2 * k].w);
            const int prim = io.hitPrim[k];
            if (prim >= 0) {
                float lam[8], beta[8];
                rload8(io.rec, slot, R_LAM, lam);
                if (d0) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) beta[i] = 1.f;
                } else {
                    rload8(io.rec, slot, R_BETA, beta);
                }
                float4 P0, P1, P2, mt;
                if (QCAP == 1 && lds_tris) {
                    P0 = g_tri1[4 * prim]; P1 = g_tri1[4 * prim + 1]; P2 = g_tri1[4 * prim + 2]; mt = g_tri1[4 * prim + 3];
                } else {
                    P0 = sc.triWorld[3 * prim]; P1 = sc.triWorld[3 * prim + 1]; P2 = sc.triWorld[3 * prim + 2];
                    // (the material table stays in global memory here: staged in LDS, CFG3 -3.5 %, r03 A/B)
                    const DevMaterial dm = sc.materials[sc.triMaterial[prim]];
                    mt = make_float4(dm.c0, dm.c1, dm.c2, dm.emit);
                }
                V3 p0 = v3(P0.x, P0.y, P0.z), p1 = v3(P1.x, P1.y, P1.z), p2 = v3(P2.x, P2.y, P2.z);
                V3 ng = vnorm(vcross(vsub(p0, p2), vsub(p1, p2)));  // Shapes.h:1073
                const float4 d4 = io.rayD[2 * k];
                V3 rayd = vnorm(v3(d4.x, d4.y, d4.z));
                if (mt.w > 0) {
                    if (io.depth == 0 && vdot(ng, rayd) < 0) {
                        float L[8];
                        rload8_or_zero(io.rec, slot, R_L, L, d0);
#pragma unroll
                        for (int i = 0; i < 8; ++i) L[i] += beta[i] * (mt.w * d65_query(sp, lam[i]));
                        rstore8(io.rec, slot, R_L, L);
                        storedL = true;
                    }
                } else if (io.depth < io.max_depth) {
                    V3 nrm = ng;
                    if (vdot(nrm, rayd) > 0) nrm = v3(-nrm.x, -nrm.y, -nrm.z);
                    const float4 hb = io.hitB[k];
                    V3 p = vadd(vadd(vmul(p0, hb.x), vmul(p1, hb.y)), vmul(p2, hb.z));
                    float off = 1e-4f * (1.0f + max3f(fabsf(p.x), fabsf(p.y), fabsf(p.z)));
                    V3 po = vadd(p, vmul(nrm, off));
                    // kLate (single leaf): both sampler draws and the geometry first, then one pass over the hero
                    // wavelengths that forms R(λ), the light term and β R per wavelength, so no R[8] array lives
                    // beside Ld[8] and β (the same operations per element; Cornell +1 %, r06_ab4; multi-level
                    // scenes keep R formed first: CFG3 −2 % with the late pass, r06_ab2)
                    constexpr bool kLate = QCAP == 1;
                    float R[8], le = 0.f, wgt = 0.f;
                    if constexpr (!kLate) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) R[i] = sigmoid_eval(mt.x, mt.y, mt.z, lam[i]);
                    }
                    Smp sm;
                    restore_sampler(ids, film, io, slot, sm, smp.kind, smp.seed);
                    // --- NEE on the quad light
                    float u0, u1;
                    sm.get2d(smp, u0, u1);
                    if (sc.n_lights > 0) {
                        const DevLight& Lq = sc.light0;
                        V3 pl = vadd(vadd(v3(Lq.p[0], Lq.p[1], Lq.p[2]), vmul(v3(Lq.e1[0], Lq.e1[1], Lq.e1[2]), u0)),
                                     vmul(v3(Lq.e2[0], Lq.e2[1], Lq.e2[2]), u1));
                        V3 wv = vsub(pl, po);
                        float dist2 = vdot(wv, wv);
                        float dist = sqrtf(dist2);
                        V3 wi = vmul(wv, 1.0f / dist);
                        float cs = vdot(nrm, wi);
                        float cl = -vdot(v3(Lq.n[0], Lq.n[1], Lq.n[2]), wi);
                        if (cs > 0 && cl > 0) {
                            le = sc.materials[Lq.material].emit;
                            float G = (cs * cl) / dist2;
                            wgt = G * Lq.area;
                            if constexpr (!kLate) {
#pragma unroll
                                for (int i = 0; i < 8; ++i)
                                    Ld[i] = ((beta[i] * (R[i] * InvPi)) * (le * d65_query(sp, lam[i]))) * wgt;
                            }
                            wantShadow = true;
                            so = po;
                            sd = wi;
                            stmax = dist * 0.999f;
                        }
                    }
                    // --- cosine-hemisphere BSDF sample (Sampling.h:449-454), frame = pbrt CoordinateSystem.  The host
                    // never traces depth max_depth in this integrator (only emitter hits could add there, and they
                    // count at depth 0 only), so the last shaded depth draws no bounce: its β, ray and sampler state
                    // would never be read.
                    if (io.depth + 1 < io.max_depth) {
                        sm.get2d(smp, u0, u1);
                        V3 wi;
                        float z;
                        if (cosine_bounce(u0, u1, nrm, wi, z)) {
                            if constexpr (!kLate) {
#pragma unroll
                                for (int i = 0; i < 8; ++i) beta[i] *= R[i];
                                rstore8(io.rec, slot, R_BETA, beta);
                            }
                            wantNext = true;
                            nO = make_float4(po.x, po.y, po.z, 0.f);
                            nD = make_float4(wi.x, wi.y, wi.z, 0.f);
                        }
                        save_sampler(io, slot, sm);
                    }
                    if constexpr (kLate) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const float Ri = sigmoid_eval(mt.x, mt.y, mt.z, lam[i]);
                            Ld[i] = ((beta[i] * (Ri * InvPi)) * (le * d65_query(sp, lam[i]))) * wgt;
                            beta[i] *= Ri;
                        }
                        if (wantNext) rstore8(io.rec, slot, R_BETA, beta);
                    }
                }
            }
        }
        // single leaf: the bounce ray leaves before the shadow ray is traced, so it is not live across the traversal
        if constexpr (QCAP == 1) {
            nO.w = __int_as_float(slot);  // the ray's origin carries its slot
            if (items.r == 1) {  // first item of the chunk
                if (wantNext) { pend[2 * threadIdx.x] = nO; pend[2 * threadIdx.x + 1] = nD; }
                pend0 = wantNext;
            } else {
                int p0, p1;
                block_append2(io.nCount, pend0, wantNext, lds, p0, p1);
                if (pend0) {
                    const float4 o0 = pend[2 * threadIdx.x], d0v = pend[2 * threadIdx.x + 1];
                    io.nO[2 * p0] = o0; io.nD[2 * p0] = d0v;
                    if (io.nkey.key) io.nkey.key[p0] = ray_sort_key(o0, d0v, io.nkey);
                }
                if (wantNext) {
                    io.nO[2 * p1] = nO; io.nD[2 * p1] = nD;
                    if (io.nkey.key) io.nkey.key[p1] = ray_sort_key(nO, nD, io.nkey);
                }
            }
        }
        if constexpr (QCAP != 1) {  // shadow queue: the ray and its pending contribution go to k_path_shadow
            if (!shq.defer) {
                int sp = WAVE ? wave_append(shq.shCount + qj * kQStride, wantShadow)
                              : block_append(shq.shCount + qj * kQStride, wantShadow, lds);
                sp += qj * io.q.S;
                if (wantShadow) {
                    shq.shO[sp] = make_float4(so.x, so.y, so.z, stmax);
                    shq.shD[sp] = make_float4(sd.x, sd.y, sd.z, __int_as_float(slot));
                    shq.shLA[sp] = make_float4(Ld[0], Ld[1], Ld[2], Ld[3]);
                    shq.shLB[sp] = make_float4(Ld[4], Ld[5], Ld[6], Ld[7]);
                    wantShadow = false;  // at depth 0 L is written as zero below; the shadow kernel adds to it
                }
            }
        }
        // NEE shadow ray, traced inline (any hit, fixed tMax) after the bounce state is written, so only the
        // pending contribution Ld stays live across the traversal.  No shadow queue in HBM.
        // Multi-level octrees: the BVH alone; a ray it cannot decide goes to the shadow queue with its pending
        // contribution (k_path_shadow runs the exact traversal and adds it in the same order).
        bool deferShadow = false;
        int hit = -1;
        if (wantShadow) {
            float b0, b1, b2, t;
            if constexpr (QCAP != 1) hit = traverse_bvh<true>(sc, 0, so, sd, stmax, b0, b1, b2, t, snn, snt, deferShadow);
            else hit = traverse_any<QCAP, true>(sc, 0, so, sd, stmax, b0, b1, b2, t, snn, snt, sfb);
        }
        if constexpr (QCAP != 1) {
            // the shadow rays the BVH could not decide: the wave resolves them one at a time with the cooperative
            // any-hit BFS (exact), so no k_path_shadow launch follows when the octree's queue bound fits its FIFO
            if (shq.defer && sc.coop_ok) {
                uint64_t am = __ballot(deferShadow);
                while (am) {
                    const int Ls = __builtin_ctzll(am);
                    am &= am - 1;
                    const V3 oL = v3(__shfl(so.x, Ls), __shfl(so.y, Ls), __shfl(so.z, Ls));
                    const V3 dL = v3(__shfl(sd.x, Ls), __shfl(sd.y, Ls), __shfl(sd.z, Ls));
                    int cp = -1;
                    float c0, c1, c2, ct;
                    ctr_t cnn = 0, cnt = 0;
                    const bool ok =
                        bfs_coop<true>(sc, 0, oL, dL, __shfl(stmax, Ls), coop_fifo_astk(), cp, c0, c1, c2, ct, cnn, cnt);
                    if (lane_id() == Ls) {
                        novf += !ok;  // (coop_ok: never; counted, C_COOPOVF)
                        hit = cp;
                        deferShadow = false;
                        ++sfb;
                        snn += cnn;
                        snt += cnt;
                    }
                }
            }
        }
        if (wantShadow && !deferShadow) {
            ++nsh;
            if (hit < 0) {
                float L[8];
                rload8_or_zero(io.rec, slot, R_L, L, d0);
#pragma unroll
                for (int i = 0; i < 8; ++i) L[i] += Ld[i];
                rstore8(io.rec, slot, R_L, L);
                storedL = true;
            }
        }
        if constexpr (QCAP != 1) {
            const int sp = wave_append(shq.shCount + qj * kQStride, deferShadow) + qj * io.q.S;
            if (deferShadow) {
                shq.shO[sp] = make_float4(so.x, so.y, so.z, stmax);
                shq.shD[sp] = make_float4(sd.x, sd.y, sd.z, __int_as_float(slot));
                shq.shLA[sp] = make_float4(Ld[0], Ld[1], Ld[2], Ld[3]);
                shq.shLB[sp] = make_float4(Ld[4], Ld[5], Ld[6], Ld[7]);
            }
        }
        if (d0 && slot >= 0 && !storedL) {
            const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            rstore8(io.rec, slot, R_L, z);
        }
        if constexpr (QCAP == 1) continue;  // (its bounce ray was appended above)
        const int pn = queue_append<WAVE>(io.nCount + qj * kQStride, wantNext, lds) + qj * io.q.S;
        if (wantNext) {
            nO.w = __int_as_float(slot);  // the ray's origin carries its slot
            io.nO[2 * pn] = nO; io.nD[2 * pn] = nD;
            if (io.nkey.key) io.nkey.key[pn] = ray_sort_key(nO, nD, io.nkey);
        }
    }
    count_add(ctr, C_SNODES, snn);
    count_add(ctr, C_STRIS, snt);
    count_add(ctr, C_SHADOW, nsh);
    count_add(ctr, C_SFALLBACK, sfb);
    if constexpr (QCAP != 1) count_add(ctr, C_COOPOVF, novf);
    if constexpr (QCAP != 1) simd_flush();
}


// Shadow-queue tracer (multi-level octrees, simple path scenes): the NEE shadow rays k_path_shade appended, traced
// with no path state live (full occupancy; DFS: depth-first any-hit, exact for a fixed tMax, §6).  An unoccluded
// ray adds its contribution to L exactly as the inline code would: per slot one shadow ray per bounce, launched
// between this bounce's shade and the next one's, so every L sees its additions in the same order.
// LEAN (every shadow ray queued, coop_ok): the BVH walk alone, the wave resolving the undecided rays with the
// cooperative any-hit BFS, as k_path_shade does inline — no per-thread BFS registers.
#ifndef RT_SHADOWQ_WAVES
#define RT_SHADOWQ_WAVES 5
#endif
template <int QCAP, bool DFS, bool LEAN = false>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(LEAN ? RT_SHADOWQ_WAVES : 1))) k_path_shadow(DevScene sc, PathIO io, ShadowQueueIO shq, unsigned long long* ctr) {
    stage_scene<QCAP>(sc, 0);
    ctr_t snn = 0, snt = 0, nsh = 0, sfb = 0, novf = 0;
    WaveTickets tk(shq.shTicket, QueueView{shq.shCount, io.q.S, 0, io.q.ns});
    int qj, base;
    while (tk.next(qj, base)) {
        if constexpr (LEAN && QCAP != 1) {
            const bool live = base + lane_id() < tk.len;
            const int k = qj * io.q.S + base + lane_id();
            float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = o4;
            int hit = -1;
            bool amb = false;
            if (live) {
                o4 = shq.shO[k];
                d4 = shq.shD[k];
                float b0, b1, b2, t;
                hit = traverse_bvh<true>(sc, 0, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z), o4.w, b0, b1, b2, t, snn,
                                         snt, amb);
            }
            uint64_t am = __ballot(live && amb);
            while (am) {
                const int Ls = __builtin_ctzll(am);
                am &= am - 1;
                const V3 oL = v3(__shfl(o4.x, Ls), __shfl(o4.y, Ls), __shfl(o4.z, Ls));
                const V3 dL = v3(__shfl(d4.x, Ls), __shfl(d4.y, Ls), __shfl(d4.z, Ls));
                int cp = -1;
                float c0 = 0.f, c1 = 0.f, c2 = 0.f, ct = 0.f;  // (any hit: only the primitive is written)
                ctr_t cnn = 0, cnt = 0;
                const bool ok = bfs_coop<true>(sc, 0, oL, dL, __shfl(o4.w, Ls), coop_fifo_astk(), cp, c0, c1, c2, ct,
                                               cnn, cnt);
                if (lane_id() == Ls) {
                    novf += !ok;  // (coop_ok: never; counted, C_COOPOVF)
                    hit = cp;
                    ++sfb;
                    snn += cnn;
                    snt += cnt;
                }
            }
            if (live) {
                ++nsh;
                if (hit < 0) {
                    const int slot = __float_as_int(d4.w);
                    const float4 la = shq.shLA[k], lb = shq.shLB[k];
                    const float Ld[8] = {la.x, la.y, la.z, la.w, lb.x, lb.y, lb.z, lb.w};
                    float L[8];
                    rload8(io.rec, slot, R_L, L);
#pragma unroll
                    for (int i = 0; i < 8; ++i) L[i] += Ld[i];
                    rstore8(io.rec, slot, R_L, L);
                }
            }
            continue;
        }
        if (base + lane_id() >= tk.len) continue;  // (reconverges at the loop latch, before the next ticket)
        const int k = qj * io.q.S + base + lane_id();
        float4 o4 = shq.shO[k], d4 = shq.shD[k];
        float b0, b1, b2, t;
        int hit = traverse_any<QCAP, true, DFS>(sc, 0, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z), o4.w, b0, b1, b2,
                                                t, snn, snt, sfb);
        ++nsh;
        if (hit < 0) {
            int slot = __float_as_int(d4.w);
            float4 la = shq.shLA[k], lb = shq.shLB[k];
            const float Ld[8] = {la.x, la.y, la.z, la.w, lb.x, lb.y, lb.z, lb.w};
            float L[8];
            rload8(io.rec, slot, R_L, L);
#pragma unroll
            for (int i = 0; i < 8; ++i) L[i] += Ld[i];
            rstore8(io.rec, slot, R_L, L);
        }
    }
    count_add(ctr, C_SNODES, snn);
    count_add(ctr, C_STRIS, snt);
    count_add(ctr, C_SHADOW, nsh);
    count_add(ctr, C_SFALLBACK, sfb);
    if constexpr (LEAN) count_add(ctr, C_COOPOVF, novf);
}

// ------------------------------------------------------------------- path mode, general scenes (§8 a21/a22)
// Same bounce as k_path_shade for scenes that need more than one quad light and Lambert triangles: analytic
// shapes, mirror and BK7/constant-eta glass (TerminateSecondary rewrites the sample's pdf), point / distant /
// disk / quad lights (one sample each, shadow rays traced inline in light order), and MIS (power heuristic).
// Semantics and sample-dimension order: oracle/rtcore.hpp LiPath, DESIGN.md §5.
template <int QCAP>
__device__ __forceinline__ bool scene_occluded(const DevScene& sc, V3 o, V3 d, float tmax, ctr_t& nn,
                                               ctr_t& nt, ctr_t& nfb) {
    float b0, b1, b2, t;
    if (traverse_any<QCAP, true>(sc, 0, o, d, tmax, b0, b1, b2, t, nn, nt, nfb) >= 0) return true;
    for (int si = 0; si < sc.n_shapes; ++si) {
        DevShape sh = ldconst(sc.shapes, si);
        V3 ph;
        float th;
        if (shape_isect(sh, o, d, tmax, ph, th)) return true;
    }
    return false;
}

// parity entry: the shadow query of the path kernels on explicit rays (d.w = tmax)
template <int QCAP>
__global__ void __launch_bounds__(kBlock) k_occluded(DevScene sc, int n, const float4* o, const float4* d, int* out,
                                                     unsigned long long* ctr) {
    ctr_t nn = 0, nt = 0, ns = 0, nfb = 0;
    stage_scene<QCAP>(sc, 0);
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        float4 o4 = o[k], d4 = d[k];
        out[k] = scene_occluded<QCAP>(sc, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z), d4.w, nn, nt, nfb) ? 1 : 0;
        ++ns;
    }
    count_add(ctr, C_SNODES, nn);
    count_add(ctr, C_STRIS, nt);
    count_add(ctr, C_SHADOW, ns);
    count_add(ctr, C_SFALLBACK, nfb);
}

// The shadow ray toward one light sample (Lights.h semantics): area lights (quad: p + u0 e1 + u1 e2;
// disk: the concentric mapping of the Disk shape) and point lights aim at the point, tMax = 0.999 dist; a distant
// light's direction is fixed (tMax = FLT_MAX; u0, u1 are drawn and unused).  k_path_shade_full evaluates it for the
// light weights and k_path_nee again for the ray: the same code on the same inputs, so the same bits.
struct LightRay {
    V3 wi;
    float tmax, dist2;
};
__device__ __forceinline__ LightRay light_ray(const DevLight& Lt, V3 po, float u0, float u1) {
    LightRay r;
    if (Lt.type == 3) {
        r.wi = v3(Lt.dir[0], Lt.dir[1], Lt.dir[2]);
        r.tmax = 3.402823466e+38f;
        r.dist2 = 1.0f;
        return r;
    }
    V3 pl;
    if (Lt.type == 0) {
        pl = vadd(vadd(v3(Lt.p[0], Lt.p[1], Lt.p[2]), vmul(v3(Lt.e1[0], Lt.e1[1], Lt.e1[2]), u0)),
                  vmul(v3(Lt.e2[0], Lt.e2[1], Lt.e2[2]), u1));
    } else if (Lt.type == 1) {
        float dx, dy;
        disk_concentric(u0, u1, dx, dy);
        pl = m4_point(Lt.o2r, v3(Lt.ro * dx, Lt.ro * dy, Lt.h));
    } else {
        pl = v3(Lt.p[0], Lt.p[1], Lt.p[2]);
    }
    const V3 wv = vsub(pl, po);
    r.dist2 = vdot(wv, wv);
    const float dist = sqrtf(r.dist2);
    r.wi = vmul(wv, 1.0f / dist);
    r.tmax = dist * 0.999f;
    return r;
}

// MC (material class): 0 every material; 1 the Lambert-or-emitter bin, 2 the mirror-or-dielectric bin (items of
// io.bin_idx: hits only: k_bin_materials appends no miss to any bin) — each bin kernel holds only its materials' code.
template <int QCAP, int MC>
#ifndef RT_FULL_WAVES
#define RT_FULL_WAVES RT_MULTI_WAVES  // the mixed-scene shade (variant builds)
#endif
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(QCAP == 1 ? 1 : RT_FULL_WAVES))) k_path_shade_full(DevScene sc, const DevSpectra* sp,
                                                                              DevSampler smp, DevFilm film,
                                                                              SampleIds ids, PathIO io,
                                                                              NeeIO nee) {
    const float InvPi = 0.31830988618379067154f;
    __shared__ int lds[kBlock / 64 + 1];
    if constexpr (MC != 2) stage_spectra(sp);  // (the mirror / glass bin reads no spectrum table)
    const bool lds_mats = stage_materials(sc);
    const int nee_f4 = nee_stride(sc.n_lights);
    // lean depth 0: k_generate stored no β = 1 / L = 0, so they start in registers and every path's L is written
    const bool d0 = io.lean && io.depth == 0;
    // multi-level octrees: per-wave tickets and appends (per-ray cost varies by 100x); single leaf: per block
    constexpr bool WAVE = QCAP != 1;
    // single leaf: the host gives the queues one shard (rt_host.cpp nsh)
    std::conditional_t<QCAP == 1, QueueItemsOne, QueueItems<WAVE>> items(io.ticket, io.q);
    int qj, qidx;
    bool live;
    while (items.next(qj, qidx, live)) {
        int k = qj * io.q.S + qidx;  // queue position (binned: of the item's hit)
        if (MC != 0 && live) k = io.bin_idx[k];
        bool wantNext = false, wantNee = false;
        unsigned neeKey = 0;
        float4 nO = make_float4(0, 0, 0, 0), nD = nO;
        int slot = -1;
        bool storedL = false;
        if (live) {
            // (one 16-B load gives the slot and the origin: binned items are scattered queue positions)
            const float4 o4 = io.rayO[2 * k];
            slot = io.depth == 0 ? k : __float_as_int(o4.w);  // (as k_path_shade)
            int prim = io.hitPrim[k];
            if (prim >= 0) {
                float lam[8], beta[8];
                rload8(io.rec, slot, R_LAM, lam);
                if (d0) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) beta[i] = 1.f;
                } else {
                    rload8(io.rec, slot, R_BETA, beta);
                }
                const float4 d4 = io.rayD[2 * k];
                V3 ro = v3(o4.x, o4.y, o4.z), rdw = v3(d4.x, d4.y, d4.z);
                V3 rayd = vnorm(rdw);
                float4 hb = io.hitB[k];
                // ---- surface (oracle SurfaceAt)
                V3 p, nrm, nout;
                bool front;
                int mid, lidx;
                if (prim < sc.n_tris) {
                    float4 P0 = sc.triWorld[3 * prim], P1 = sc.triWorld[3 * prim + 1], P2 = sc.triWorld[3 * prim + 2];
                    V3 p0 = v3(P0.x, P0.y, P0.z), p1 = v3(P1.x, P1.y, P1.z), p2 = v3(P2.x, P2.y, P2.z);
                    V3 ng = vnorm(vcross(vsub(p0, p2), vsub(p1, p2)));
                    p = vadd(vadd(vmul(p0, hb.x), vmul(p1, hb.y)), vmul(p2, hb.z));
                    nout = ng;
                    front = vdot(ng, rayd) < 0;
                    nrm = ng;
                    if (vdot(nrm, rayd) > 0) nrm = v3(-ng.x, -ng.y, -ng.z);
                    mid = sc.triMaterial[prim];
                    lidx = mat_at(sc, lds_mats, mid).light;
                } else {
                    const DevShape& s = sc.shapes[prim - sc.n_tris];
                    V3 rdo = vnorm(m4_dir(s.r2o, rdw));
                    V3 ph = v3(hb.x, hb.y, hb.z);
                    V3 no = shape_normal_obj(s, ph);
                    bool flip = vdot(no, rdo) > 0;
                    if (flip) no = v3(-no.x, -no.y, -no.z);
                    V3 nw = vnorm(m3_mul(s.n2r, no));
                    p = m4_point(s.o2r, ph);
                    nrm = nw;
                    front = !flip;
                    nout = flip ? v3(-nw.x, -nw.y, -nw.z) : nw;
                    mid = s.material;
                    lidx = s.light;
                }
                const DevMaterial mt = mat_at(sc, lds_mats, mid);
                // R_MISC (dimension, prevPdf, TerminateSecondary flag) read once and written back once, as a float4:
                // the record is slot-indexed, so every narrow access of a wave is 64 scattered requests
                float4 misc = *recf(io.rec, slot, R_MISC);
                const float prevPdf = misc.y;
                if (MC != 2 && mt.emit > 0) {  // one-sided pure emitter, ends the path
                    if (front) {
                        float L[8];
                        rload8_or_zero(io.rec, slot, R_L, L, d0);
                        if (prevPdf == 0) {
#pragma unroll
                            for (int i = 0; i < 8; ++i) L[i] += beta[i] * (mt.emit * d65_query(sp, lam[i]));
                        } else if (sc.mis && lidx >= 0) {
                            const DevLight& Lt = sc.lights[lidx];
                            V3 dv = vsub(p, ro);
                            float dist2 = vdot(dv, dv);
                            float cl = -vdot(v3(Lt.n[0], Lt.n[1], Lt.n[2]), rayd);
                            if (cl > 0) {
                                float wb = power_heuristic(prevPdf, dist2 / (cl * Lt.area));
#pragma unroll
                                for (int i = 0; i < 8; ++i)
                                    L[i] += (beta[i] * (mt.emit * d65_query(sp, lam[i]))) * wb;
                            }
                        }
                        rstore8(io.rec, slot, R_L, L);
                        storedL = true;
                    }
                } else if (io.depth < io.max_depth) {
                    float off = 1e-4f * (1.0f + max3f(fabsf(p.x), fabsf(p.y), fabsf(p.z)));
                    float R[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) R[i] = sigmoid_eval(mt.c0, mt.c1, mt.c2, lam[i]);
                    if (MC != 1 && mt.type == 1) {  // perfect mirror: no sampler draws
#pragma unroll
                        for (int i = 0; i < 8; ++i) beta[i] *= R[i];
                        rstore8(io.rec, slot, R_BETA, beta);
                        V3 po = vadd(p, vmul(nrm, off)), wi = reflect_dir(rayd, nrm);
                        wantNext = true;
                        nO = make_float4(po.x, po.y, po.z, 0.f);
                        nD = make_float4(wi.x, wi.y, wi.z, 0.f);
                        misc.y = 0.f;
                        *recf(io.rec, slot, R_MISC) = misc;
                    } else {
                        Smp sm;
                        restore_sampler(ids, film, io, slot, sm, smp.kind, smp.seed, __float_as_int(misc.x),
                                        __float_as_int(misc.w));
                        if (MC != 1 && mt.type == 2) {  // smooth dielectric
                            if (mt.eta == 0) {  // dispersive BK7: TerminateSecondary (spectrum.h:302-310)
                                if (io.lean == 2) {  // the pdfs are not stored: flag it, k_path_film divides
                                    misc.z = 1.f;
                                } else {
                                    float pdf[8];
                                    load8(io.pdfA, io.pdfB, slot, pdf);
                                    bool term = true;
#pragma unroll
                                    for (int i = 1; i < 8; ++i) term = term && pdf[i] == 0;
                                    if (!term) {
#pragma unroll
                                        for (int i = 1; i < 8; ++i) pdf[i] = 0;
                                        pdf[0] /= 8;
                                        store8(io.pdfA, io.pdfB, slot, pdf);
                                    }
                                }
                            }
                            float eta = mt.eta != 0 ? mt.eta : piecewise_query(sp->bk7_lambda, sp->bk7_value, sp->bk7_n, lam[0]);
                            float u = sm.get1d(smp);
                            V3 wo = v3(-rayd.x, -rayd.y, -rayd.z);
                            float Fr = fr_dielectric(vdot(nout, wo), eta);
                            V3 wt, po, wi;
                            float etap;
                            if (u < Fr || !refract_dir(wo, nout, eta, etap, wt)) {
                                po = vadd(p, vmul(nrm, off));
                                wi = reflect_dir(rayd, nrm);
                                if (d0) rstore8(io.rec, slot, R_BETA, beta);  // (lean: β = 1 was never stored)
                            } else {
#pragma unroll
                                for (int i = 0; i < 8; ++i) beta[i] /= (etap * etap);
                                rstore8(io.rec, slot, R_BETA, beta);
                                po = vsub(p, vmul(nrm, off));
                                wi = wt;
                            }
                            wantNext = true;
                            nO = make_float4(po.x, po.y, po.z, 0.f);
                            nD = make_float4(wi.x, wi.y, wi.z, 0.f);
                            misc.y = 0.f;
                        } else if constexpr (MC != 2) {  // Lambert: NEE per light (k_path_nee), then a cosine bounce
                            V3 po = vadd(p, vmul(nrm, off));
                            float4* nr = nee.rec + (size_t)slot * nee_f4;
                            float* nuv = reinterpret_cast<float*>(nr + N_UV);
                            float* nwgt = nuv + 4 * ((sc.n_lights + 1) / 2);
                            if (nee.key) neeKey = morton_key(po.x, po.y, po.z, nee.lo, nee.scale, nee.key_bits);
                            // the record is written in whole float4s (two lights' samples, four lights' weights per
                            // store) instead of one 4-B store per value: 4 stores per vertex instead of 13 with 4 lights
                            float pu0 = 0.f, pu1 = 0.f, w0 = 0.f, w1 = 0.f, w2 = 0.f, w3 = 0.f;
                            const int nl = sc.n_lights;
                            for (int li = 0; li < nl; ++li) {
                                const DevLight Lt = ldconst(sc.lights, li);
                                float u0, u1;
                                sm.get2d(smp, u0, u1);
                                const LightRay lr = light_ray(Lt, po, u0, u1);
                                const float cs = vdot(nrm, lr.wi);
                                bool ok;
                                float wgt;
                                if (Lt.type <= 1) {
                                    float cl = -vdot(v3(Lt.n[0], Lt.n[1], Lt.n[2]), lr.wi);
                                    ok = cs > 0 && cl > 0;
                                    float G = (cs * cl) / lr.dist2;
                                    wgt = G * Lt.area;
                                    if (sc.mis) wgt = wgt * power_heuristic(lr.dist2 / (cl * Lt.area), cs * InvPi);
                                } else {
                                    ok = cs > 0;
                                    wgt = cs * (Lt.type == 2 ? 1.0f / lr.dist2 : 1.0f);
                                }
                                const float wv = ok ? wgt : -1.0f;  // (an accepted light's weight is >= 0 or NaN)
                                const int l4 = li & 3;
                                w0 = l4 == 0 ? wv : w0;
                                w1 = l4 == 1 ? wv : w1;
                                w2 = l4 == 2 ? wv : w2;
                                w3 = l4 == 3 ? wv : w3;
                                if ((li & 1) || li + 1 == nl)
                                    reinterpret_cast<float4*>(nuv)[li >> 1] =
                                        (li & 1) ? make_float4(pu0, pu1, u0, u1) : make_float4(u0, u1, 0.f, 0.f);
                                pu0 = u0;
                                pu1 = u1;
                                if (l4 == 3 || li + 1 == nl) reinterpret_cast<float4*>(nwgt)[li >> 2] = make_float4(w0, w1, w2, w3);
                                wantNee = wantNee || ok;
                            }
                            // cosine-hemisphere bounce (Sampling.h:449-454), pbrt CoordinateSystem frame
                            float u0, u1;
                            sm.get2d(smp, u0, u1);
                            V3 wi;
                            float z;
                            const bool bounced = cosine_bounce(u0, u1, nrm, wi, z);
                            if (bounced) {
                                if (!wantNee) {  // (with NEE, k_path_nee forms β R after the light terms)
#pragma unroll
                                    for (int i = 0; i < 8; ++i) beta[i] *= R[i];
                                    rstore8(io.rec, slot, R_BETA, beta);
                                }
                                wantNext = true;
                                nO = make_float4(po.x, po.y, po.z, 0.f);
                                nD = make_float4(wi.x, wi.y, wi.z, 0.f);
                                misc.y = z * InvPi;
                            }
                            if (wantNee)
                                nr[N_PO] = make_float4(po.x, po.y, po.z,
                                                       __uint_as_float((unsigned)mid | (bounced ? 0x80000000u : 0u)));
                        }
                        save_sampler(io, slot, sm, io.dim >= 0);
                        if (io.dim < 0) misc.x = __int_as_float(sm.dim);
                        *recf(io.rec, slot, R_MISC) = misc;
                    }
                }
            }
        }
        if (d0 && slot >= 0 && !storedL) {  // (k_path_nee and the film read it; misses: k_bin_materials or here)
            const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            rstore8(io.rec, slot, R_L, z);
        }
        if constexpr (MC != 2) {
            const int pe = queue_append<WAVE>(nee.len + qj * kQStride, wantNee, lds) + qj * io.q.S;
            if (wantNee) {
                nee.slot[pe] = slot;
                if (nee.key) nee.key[pe] = neeKey;
            }
        }
        const int pn = queue_append<WAVE>(io.nCount + qj * kQStride, wantNext, lds) + qj * io.q.S;
        if (wantNext) {
            nO.w = __int_as_float(slot);  // the ray's origin carries its slot
            io.nO[2 * pn] = nO; io.nD[2 * pn] = nD;
            if (io.nkey.key) io.nkey.key[pn] = ray_sort_key(nO, nD, io.nkey);
        }
    }
}

// Deferred NEE (NeeIO): per queued Lambert vertex, the shadow rays of its lights in light order (any hit, fixed
// tMax, then the analytic shapes: scene_occluded), then L += ((x (Le D65(λ))) wgt) for the visible lights in the
// same order — the inline loop's arithmetic term for term.  Only the shadow rays and L are live here.
// scene_occluded over the BVH alone (multi-level octrees): amb = the canonical rule could not decide
__device__ __forceinline__ bool shapes_occluded(const DevScene& sc, V3 o, V3 d, float tmax) {
    for (int si = 0; si < sc.n_shapes; ++si) {
        DevShape sh = ldconst(sc.shapes, si);
        V3 ph;
        float th;
        if (shape_isect(sh, o, d, tmax, ph, th)) return true;
    }
    return false;
}
__device__ __forceinline__ bool scene_occluded_bvh(const DevScene& sc, V3 o, V3 d, float tmax, ctr_t& nn, ctr_t& nt,
                                                   bool& amb) {
    float b0, b1, b2, t;
    if (traverse_bvh<true>(sc, 0, o, d, tmax, b0, b1, b2, t, nn, nt, amb) >= 0) return true;
    if (amb) return false;
    return shapes_occluded(sc, o, d, tmax);
}

// parity entry (RTMI_DEBUG_PATH_KERNELS, multi-level scenes with coop_ok): the shadow query as the path kernels run
// it — the BVH walk, the wave-cooperative any-hit BFS for the rays it cannot decide, then the analytic shapes
// (k_path_nee's per-light test; k_path_shade's inline test is the same without shapes) — one ray per lane, whole waves
template <int QCAP>
__global__ void __launch_bounds__(kBlock) k_occluded_path(DevScene sc, int n, const float4* o, const float4* d,
                                                          int* out, unsigned long long* ctr) {
    ctr_t nn = 0, nt = 0, ns = 0, nfb = 0, novf = 0;
    stage_scene<QCAP>(sc, 0);
    const int nw = (int)(gridDim.x * (blockDim.x >> 6));
    for (int base = ((int)blockIdx.x * (int)(blockDim.x >> 6) + (int)(threadIdx.x >> 6)) * 64; base < n; base += nw * 64) {
        const int k = base + lane_id();
        const bool live = k < n;
        float4 o4 = make_float4(0.f, 0.f, 0.f, 0.f), d4 = o4;
        bool occ = false, amb = false;
        if (live) {
            o4 = o[k];
            d4 = d[k];
            occ = scene_occluded_bvh(sc, v3(o4.x, o4.y, o4.z), v3(d4.x, d4.y, d4.z), d4.w, nn, nt, amb);
        }
        uint64_t am = __ballot(live && amb);
        while (am) {
            const int Ls = __builtin_ctzll(am);
            am &= am - 1;
            const V3 oL = v3(__shfl(o4.x, Ls), __shfl(o4.y, Ls), __shfl(o4.z, Ls));
            const V3 dL = v3(__shfl(d4.x, Ls), __shfl(d4.y, Ls), __shfl(d4.z, Ls));
            int cp = -1;
            float c0 = 0.f, c1 = 0.f, c2 = 0.f, ct = 0.f;
            ctr_t cnn = 0, cnt = 0;
            const bool ok = bfs_coop<true>(sc, 0, oL, dL, __shfl(d4.w, Ls), coop_fifo_astk(), cp, c0, c1, c2, ct, cnn, cnt);
            if (lane_id() == Ls) {
                novf += !ok;
                occ = cp >= 0 || shapes_occluded(sc, oL, dL, d4.w);
                ++nfb;
                nn += cnn;
                nt += cnt;
            }
        }
        if (live) {
            out[k] = occ ? 1 : 0;
            ++ns;
        }
    }
    count_add(ctr, C_SNODES, nn);
    count_add(ctr, C_STRIS, nt);
    count_add(ctr, C_SHADOW, ns);
    count_add(ctr, C_SFALLBACK, nfb);
    count_add(ctr, C_COOPOVF, novf);
}

// FB = false: the NEE queue.  On multi-level octrees a vertex with a shadow ray the BVH alone cannot decide is not
// accumulated but listed (nee.fb_slot); FB = true then re-runs the listed vertices with the exact traversal (the
// reference BFS for the ambiguous rays), so this kernel never holds the BFS's registers (128 VGPRs + spill -> 108).
// A vertex's lights are always accumulated together, in light order, by one of the two.
template <int QCAP, bool FB>
#ifndef RT_NEE_WAVES
#define RT_NEE_WAVES 4  // (variant builds: Makefile `variants`)
#endif
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(QCAP == 1 ? 1 : (FB ? 2 : RT_NEE_WAVES)))) k_path_nee(DevScene sc, const DevSpectra* sp, PathIO io,
                                                                       NeeIO nee, unsigned long long* ctr) {
    stage_spectra(sp);
    stage_scene<QCAP>(sc, 0);
    ctr_t snn = 0, snt = 0, nsh = 0, sfb = 0, nvx = 0, novf = 0;
    const int nl = sc.n_lights, nf4 = nee_stride(nl);
    // one path vertex: visibility of each sampled light, then the unoccluded lights' contributions in order, then
    // the throughput of the continued path (NeeIO)
    const float InvPi = 0.31830988618379067154f;
    const int nuv4 = (nl + 1) / 2;
    // COOP (multi-level NEE queue): every lane of the wave calls vertex() in step (live = it has a vertex), so the
    // light loop reconverges after each light and the wave resolves the shadow rays the BVH could not decide with the
    // cooperative any-hit BFS (exact) instead of listing their vertices for k_path_nee<Q, true> (no fallback launch
    // when the octree's queue bound fits its FIFO, DevScene coop_ok)
    constexpr bool COOP = QCAP != 1 && !FB;
    auto vertex = [&](int slot, bool live) __attribute__((always_inline)) {
        const float4* r = nee.rec + (size_t)(live ? slot : 0) * nf4;  // (not live: slot 0's record, unused)
        const float4 p4 = r[N_PO];
        const V3 po = v3(p4.x, p4.y, p4.z);
        const unsigned tag = __float_as_uint(p4.w);
        const float* uv = reinterpret_cast<const float*>(r + N_UV);
        const float* wg = uv + 4 * nuv4;
        // the sampled lights (weight >= 0; < 0: not sampled, cos <= 0) as a bit mask, from the weights read four per
        // 16-B load up front instead of one 4-B load at the top of every light's iteration
        uint64_t wmask = 0;
        for (int q = 0; q < (nl + 3) >> 2; ++q) {
            const float4 w4 = reinterpret_cast<const float4*>(wg)[q];
            wmask |= (uint64_t)((w4.x >= 0.f ? 1u : 0u) | (w4.y >= 0.f ? 2u : 0u) | (w4.z >= 0.f ? 4u : 0u) |
                                (w4.w >= 0.f ? 8u : 0u)) << (4 * q);
        }
        uint64_t vis = 0;
        ctr_t nv = 0;
        bool defer = false;
        for (int li = 0; li < nl; ++li) {
            const bool act = live && !defer && ((wmask >> li) & 1u);
            bool occ = false, amb = false;
            LightRay lr{};
            if (act) {
                ++nv;
                lr = light_ray(ldconst(sc.lights, li), po, uv[2 * li], uv[2 * li + 1]);
                if constexpr (COOP) occ = scene_occluded_bvh(sc, po, lr.wi, lr.tmax, snn, snt, amb);
                else occ = scene_occluded<QCAP>(sc, po, lr.wi, lr.tmax, snn, snt, sfb);
            }
            if constexpr (COOP) {
                if (sc.coop_ok) {
                    uint64_t am = __ballot(amb);
                    while (am) {
                        const int Ls = __builtin_ctzll(am);
                        am &= am - 1;
                        const V3 oL = v3(__shfl(po.x, Ls), __shfl(po.y, Ls), __shfl(po.z, Ls));
                        const V3 dL = v3(__shfl(lr.wi.x, Ls), __shfl(lr.wi.y, Ls), __shfl(lr.wi.z, Ls));
                        int cp = -1;
                        float c0, c1, c2, ct;
                        ctr_t cnn = 0, cnt = 0;
                        const bool ok = bfs_coop<true>(sc, 0, oL, dL, __shfl(lr.tmax, Ls), coop_fifo_astk(), cp, c0,
                                                       c1, c2, ct, cnn, cnt);
                        if (lane_id() == Ls) {  // the octree's answer, then the analytic shapes (scene_occluded_bvh)
                            novf += !ok;        // (coop_ok: never; counted, C_COOPOVF)
                            occ = cp >= 0 || shapes_occluded(sc, po, lr.wi, lr.tmax);
                            amb = false;
                            ++sfb;
                            snn += cnn;
                            snt += cnt;
                        }
                    }
                }
                if (amb) defer = true;  // (coop_ok == 0: the vertex goes to k_path_nee<Q, true>)
            }
            if (act && !defer && !occ) vis |= 1ull << li;
        }
        if (!live) return;
        if (defer) {  // (rare: vector atomics per lane)
            nee.fb_slot[atomicAdd(nee.fb_len, 1)] = slot;
            return;
        }
        nsh += nv;
        nvx += 1;
        const bool bounced = (tag >> 31) != 0;
        if (vis || bounced) {
            float lam[8], beta[8], R[8];
            rload8(io.rec, slot, R_LAM, lam);
            if (io.lean && io.depth == 0) {  // (lean depth 0: β = 1, never stored)
#pragma unroll
                for (int i = 0; i < 8; ++i) beta[i] = 1.f;
            } else {
                rload8(io.rec, slot, R_BETA, beta);
            }
            const DevMaterial mt = sc.materials[tag & 0x7fffffffu];
#pragma unroll
            for (int i = 0; i < 8; ++i) R[i] = sigmoid_eval(mt.c0, mt.c1, mt.c2, lam[i]);
            if (vis) {
                float L[8], x[8];
                rload8(io.rec, slot, R_L, L);
#pragma unroll
                for (int i = 0; i < 8; ++i) x[i] = beta[i] * (R[i] * InvPi);
                float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f);  // the weights again, four per 16-B load
                int wq = -1;
                for (int li = 0; li < nl; ++li) {
                    if (!((vis >> li) & 1)) continue;
                    const DevLight Lt = ldconst(sc.lights, li);
                    const float sc_le = Lt.type <= 1 ? sc.materials[Lt.material].emit : Lt.scale;
                    if ((li >> 2) != wq) {
                        wq = li >> 2;
                        w4 = reinterpret_cast<const float4*>(wg)[wq];
                    }
                    const int l4 = li & 3;
                    const float wgt = l4 == 0 ? w4.x : l4 == 1 ? w4.y : l4 == 2 ? w4.z : w4.w;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        float Le = sc_le * d65_query(sp, lam[i]);
                        L[i] += ((x[i] * Le)) * wgt;
                    }
                }
                rstore8(io.rec, slot, R_L, L);
            }
            if (bounced) {
#pragma unroll
                for (int i = 0; i < 8; ++i) beta[i] *= R[i];
                rstore8(io.rec, slot, R_BETA, beta);
            }
        }
    };
    if constexpr (FB) {
        const int n = *nee.fb_len;
        for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
            vertex(nee.fb_slot[k], true);
    } else {
        const QueueView q{nee.len, io.q.S, 0, io.q.ns};
        std::conditional_t<QCAP == 1, QueueItemsOne, QueueItems<QCAP != 1>> items(nee.ticket, q);
        int qj, qidx;
        bool live;
        while (items.next(qj, qidx, live)) {
            if constexpr (COOP) {  // (wave tickets: the wave's lanes step together)
                vertex(live ? nee.slot[qj * q.S + qidx] : 0, live);
            } else {
                if (!live) continue;  // (no block-level synchronisation in this kernel)
                vertex(nee.slot[qj * q.S + qidx], true);
            }
        }
    }
    count_add(ctr, C_SNODES, snn);
    count_add(ctr, C_STRIS, snt);
    count_add(ctr, C_SHADOW, nsh);
    count_add(ctr, C_SFALLBACK, sfb);
    count_add(ctr, C_NEEVTX, nvx);
    if constexpr (QCAP != 1) count_add(ctr, C_COOPOVF, novf);
    if constexpr (QCAP != 1 && !FB) simd_flush();
}

// sensor + film for path mode (pixel-owned, index order)
__global__ void __launch_bounds__(kBlock) k_path_film(const DevSpectra* sp, DevFilm film, PathFilmIO io,
                                                      unsigned long long* ctr) {
    stage_spectra(sp);
    if (io.lean) stage_warp_tables();  // (block-uniform)
    ctr_t ns = 0;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < io.n_pixels; j += gridDim.x * blockDim.x) {
        int pixel = io.work_pixels[j];
        float4 f = io.film[pixel];
        for (int i = 0; i < io.n_index; ++i) {
            int s = i * io.n_pixels + j;
            float lam[8], pdf[8], L[8], rgb[3];
            rload8(io.rec, s, R_LAM, lam);
            if (io.lean) {
#pragma unroll
                for (int w = 0; w < 8; ++w) pdf[w] = visible_pdf<WarpTab>(lam[w]);  // the value k_generate would have stored
                if (io.lean == 2 && recf(io.rec, s, R_MISC)->z != 0.f) {  // TerminateSecondary (spectrum.h:302-310)
#pragma unroll
                    for (int w = 1; w < 8; ++w) pdf[w] = 0;
                    pdf[0] /= 8;
                }
            } else {
                load8(io.pdfA, io.pdfB, s, pdf);
            }
            rload8(io.rec, s, R_L, L);
            to_sensor_rgb_spk(sp, L, lam, pdf, film.imaging_ratio, rgb);
            const float w = 1.0f;
            f.x += w * gclamp(rgb[0], 0.0f, 1.0f);
            f.y += w * gclamp(rgb[1], 0.0f, 1.0f);
            f.z += w * gclamp(rgb[2], 0.0f, 1.0f);
            f.w += w;
            ++ns;
        }
        io.film[pixel] = f;
    }
    count_add(ctr, C_SAMPLES, ns);
}

// a20 resolve (RayTracerTestApp.h:437-451): rgbsum/weightsum → XYZFromSensorRGB → RGBFromXYZ → clamp → u8
// pbrt ColorEncoding::sRGB LinearToSRGB8 (color.h:537-557): EvaluatePolynomial is a Horner chain of FMAs
__device__ __forceinline__ unsigned char linear_to_srgb8(float v) {
    if (v <= 0) return 0;
    if (v >= 1) return 255;
    float e;
    if (v <= 0.0031308f) {
        e = 12.92f * v;
    } else {
        float s = sqrtf(v);
        float p = __builtin_fmaf(s, __builtin_fmaf(s, __builtin_fmaf(s, __builtin_fmaf(s, __builtin_fmaf(s,
                  -0.016202083165206348f, 0.7551545191665577f), 2.0041169284241644f), 0.7642611304733891f),
                  0.03453868659826638f), -0.0016829072605308378f);
        float q = __builtin_fmaf(s, __builtin_fmaf(s, __builtin_fmaf(s, __builtin_fmaf(s, __builtin_fmaf(s, 1.f,
                  1.8970238036421054f), 0.6085338522168684f), 0.03467195408529984f), -0.00004375359692957097f),
                  4.178892964897981e-7f);
        e = p / q * v;
    }
    float r = roundf(255.f * e);
    return (unsigned char)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

__global__ void k_resolve(int n, const float4* film, const float* __restrict__ A, const float* __restrict__ B,
                          unsigned char* out, int srgb) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 f = film[i];
    float s0 = f.x / f.w, s1 = f.y / f.w, s2 = f.z / f.w;
    float x[3], r[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) x[k] = (A[0 * 3 + k] * s0 + A[1 * 3 + k] * s1) + A[2 * 3 + k] * s2;
#pragma unroll
    for (int k = 0; k < 3; ++k) r[k] = (B[0 * 3 + k] * x[0] + B[1 * 3 + k] * x[1]) + B[2 * 3 + k] * x[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (srgb) {
            out[3 * i + k] = r[k] == r[k] ? linear_to_srgb8(gclamp(r[k], 0.0f, 1.0f)) : 0;
        } else {
            float v = 255.0f * gclamp(r[k], 0.0f, 1.0f);
            out[3 * i + k] = (v == v) ? (unsigned char)v : 0;
        }
    }
}

// ========================================================== multi-device film exchange
// Owned-pixel gather / scatter between a film and a compact buffer in the shard's work order: the only data a
// device of a multi-GPU context sends or receives per pass.  Pure copies (no arithmetic), so the exchanged film is
// bit-identical to a one-device render.
__global__ void __launch_bounds__(kBlock) k_film_gather(int n, const int* __restrict__ work, const float4* __restrict__ film,
                                                        float4* __restrict__ out) {
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) out[k] = film[work[k]];
}
__global__ void __launch_bounds__(kBlock) k_film_scatter(int n, const int* __restrict__ work, const float4* __restrict__ in,
                                                         float4* __restrict__ film) {
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) film[work[k]] = in[k];
}

// ============================================================================== launch wrappers
// The fallback passes (the few rays the BVH alone could not decide: 0-100 per launch on CFG3/CFG4) run on a small
// grid, so their launch neither waits for nor occupies the whole GPU (a resident grid there: CFG3 +0.9 % instead of
// the BFS-free kernels' full gain).
static constexpr int kFallbackBlocks = 64;
static inline int grid_for(int n, int grid) {
    int g = (n + kBlock - 1) / kBlock;
    if (grid > 0 && g > grid) g = grid;
    return g < 1 ? 1 : g;
}

// Persistent grid-stride kernels: every block gets the same share of the queue, so launching more blocks than can
// be resident at once (grid = 8 per CU, occupancy 4-5 per CU) runs a second, under-occupied round of blocks.  The
// grid is clamped to exactly the resident block count of the kernel (`grid` is CUs x 8; Cornell 1112 -> 1202).
template <class F>
static int resident_grid(F kern, int gb, int grid) {
    static std::mutex mu;
    static std::unordered_map<const void*, int> cache;
    int per_cu = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find((const void*)kern);
        if (it == cache.end()) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, 0) != hipSuccess) per_cu = 0;
            cache[(const void*)kern] = per_cu;
        } else {
            per_cu = it->second;
        }
    }
    if (per_cu > 0) {
        int res = per_cu * (grid / 8);
        if (res > 0 && gb > res) gb = res;
    }
    return gb;
}

hipError_t launch_emitter_filter(hipStream_t st, int grid, const DevScene& sc, const EmitIO& io) {
    if (sc.n_emit_tris < 0 || sc.n_emit_tris > kMaxEmitTris) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_emitter_filter, dim3(grid_for(io.q.n ? io.q.n : grid * kBlock, grid)), dim3(kBlock), 0, st,
                       sc, io);
    return hipGetLastError();
}

hipError_t launch_generate(hipStream_t st, int grid, int nS, const SampleIds& ids, const DevCamera& cam,
                           const DevSampler& smp, const DevFilm& film, const GenOut& out) {
    hipLaunchKernelGGL(k_generate, dim3(grid_for(nS, grid)), dim3(kBlock), 0, st, nS, ids, cam, smp, film, out);
    return hipGetLastError();
}

hipError_t launch_trace_closest(hipStream_t st, int grid, int qcap, const DevScene& sc, const TraceIO& io,
                                unsigned long long* ctr) {
    int gb = grid_for(io.q.len ? grid * kBlock : io.q.n, grid);
    if (qcap == 0) gb = std::min(gb, sc.ring_threads / kBlock);  // one ring per resident thread
    dim3 b(kBlock);
    const bool fbl = io.fb_pos != nullptr;
    if (fbl && (!io.fb_len || qcap == 1)) return hipErrorInvalidValue;
#define RT_TRACE_CASE(Q)                                                                                          \
    case Q:                                                                                                       \
        if (fbl)                                                                                                  \
            hipLaunchKernelGGL((k_trace_closest<Q, true>), dim3(resident_grid(k_trace_closest<Q, true>, gb, grid)), b, \
                               0, st, sc, io, ctr);                                                               \
        else                                                                                                      \
            hipLaunchKernelGGL((k_trace_closest<Q, false>), dim3(resident_grid(k_trace_closest<Q, false>, gb, grid)), \
                               b, 0, st, sc, io, ctr);                                                            \
        break;
    switch (qcap) {
        RT_TRACE_CASE(0)
        case 1: hipLaunchKernelGGL((k_trace_closest<1, false>), dim3(resident_grid(k_trace_closest<1, false>, gb, grid)), b, 0, st, sc, io, ctr); break;
        RT_TRACE_CASE(16)
        default: return hipErrorInvalidValue;
    }
#undef RT_TRACE_CASE
    return hipGetLastError();
}

hipError_t launch_trace_fallback(hipStream_t st, int grid, int qcap, const DevScene& sc, const TraceIO& io,
                                 unsigned long long* ctr) {
    if (!io.fb_pos || !io.fb_len) return hipErrorInvalidValue;
    int gb = std::min(grid > 0 ? grid : 1, kFallbackBlocks);
    if (qcap == 0) gb = std::min(gb, sc.ring_threads / kBlock);  // one ring per resident thread
    dim3 b(kBlock);
    switch (qcap) {
        case 0: hipLaunchKernelGGL(k_trace_fallback<0>, dim3(resident_grid(k_trace_fallback<0>, gb, grid)), b, 0, st, sc, io, ctr); break;
        case 16: hipLaunchKernelGGL(k_trace_fallback<16>, dim3(resident_grid(k_trace_fallback<16>, gb, grid)), b, 0, st, sc, io, ctr); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_ref_shade_film(hipStream_t st, int grid, const DevScene& sc, const DevSpectra* sp, const DevFilm& film,
                                 const ShadeRefIO& io, unsigned long long* ctr) {
    hipLaunchKernelGGL(k_ref_shade_film, dim3(grid_for(io.n_pixels, grid)), dim3(kBlock), 0, st, sc, sp, film, io, ctr);
    return hipGetLastError();
}

hipError_t launch_records(hipStream_t st, const DevScene& sc, const DevSpectra* sp, const DevFilm& film,
                          const ShadeRefIO& sio, const RecordIO& io) {
    hipLaunchKernelGGL(k_records, dim3(grid_for(io.n, 0)), dim3(kBlock), 0, st, sc, sp, film, sio, io);
    return hipGetLastError();
}


hipError_t launch_path_shadow(hipStream_t st, int grid, int qcap, bool dfs, const DevScene& sc, const PathIO& io,
                              const ShadowQueueIO& shq, unsigned long long* ctr) {
    int gb = grid > 0 ? grid : 1;
    if (shq.defer) gb = std::min(gb, kFallbackBlocks);
    if (qcap == 0) gb = std::min(gb, sc.ring_threads / kBlock);  // one ring per resident thread
    dim3 b(kBlock);
#define RT_SHADOW_CASE(Q)                                                                                        \
    case Q:                                                                                                      \
        if (!shq.defer && sc.coop_ok)                                                                            \
            hipLaunchKernelGGL((k_path_shadow<Q, false, true>), dim3(resident_grid(k_path_shadow<Q, false, true>, gb, grid)), \
                               b, 0, st, sc, io, shq, ctr);                                                           \
        else if (dfs)                                                                                            \
            hipLaunchKernelGGL((k_path_shadow<Q, true>), dim3(resident_grid(k_path_shadow<Q, true>, gb, grid)), b, \
                               0, st, sc, io, shq, ctr);                                                              \
        else                                                                                                     \
            hipLaunchKernelGGL((k_path_shadow<Q, false>), dim3(resident_grid(k_path_shadow<Q, false>, gb, grid)), \
                               b, 0, st, sc, io, shq, ctr);                                                           \
        break;
    switch (qcap) {
        RT_SHADOW_CASE(0)
        RT_SHADOW_CASE(16)
        default: return hipErrorInvalidValue;
    }
#undef RT_SHADOW_CASE
    return hipGetLastError();
}

hipError_t launch_path_shade(hipStream_t st, int grid, int qcap, const DevScene& sc, const DevSpectra* sp,
                             const DevSampler& smp, const DevFilm& film, const SampleIds& ids, const PathIO& io,
                             unsigned long long* ctr, const ShadowQueueIO& shq, const NeeIO& nee, int matclass) {
    int gb = grid > 0 ? grid : 1;
    if (qcap == 0) gb = std::min(gb, sc.ring_threads / kBlock);  // one ring per resident thread
    dim3 b(kBlock);
    if (sc.full && sc.n_lights > 0 && !nee.rec) return hipErrorInvalidValue;  // NEE records are required
    if (!sc.full && qcap != 1 && !shq.shO) return hipErrorInvalidValue;       // so is the shadow queue
#define RT_SHADE_CASE(Q)                                                                                         \
    case Q:                                                                                                      \
        if (sc.full && Q != 1 && matclass == 1)                                                                 \
            hipLaunchKernelGGL((k_path_shade_full<Q, 1>), dim3(resident_grid(k_path_shade_full<Q, 1>, gb, grid)), b, 0, \
                               st, sc, sp, smp, film, ids, io, nee);                                             \
        else if (sc.full && Q != 1 && matclass == 2)                                                            \
            hipLaunchKernelGGL((k_path_shade_full<Q, 2>), dim3(resident_grid(k_path_shade_full<Q, 2>, gb, grid)), b, 0, \
                               st, sc, sp, smp, film, ids, io, nee);                                             \
        else if (sc.full)                                                                                        \
            hipLaunchKernelGGL((k_path_shade_full<Q, 0>), dim3(resident_grid(k_path_shade_full<Q, 0>, gb, grid)), b, 0, \
                               st, sc, sp, smp, film, ids, io, nee);                                             \
        else                                                                                                     \
            hipLaunchKernelGGL(k_path_shade<Q>, dim3(resident_grid(k_path_shade<Q>, gb, grid)), b, 0, st, sc, sp,  \
                               smp, film, ids, io, ctr, shq);                                                    \
        break;
    switch (qcap) {
        RT_SHADE_CASE(0)
        RT_SHADE_CASE(1)
        RT_SHADE_CASE(16)
        default: return hipErrorInvalidValue;
    }
#undef RT_SHADE_CASE
    return hipGetLastError();
}

hipError_t launch_path_nee(hipStream_t st, int grid, int qcap, const DevScene& sc, const DevSpectra* sp,
                           const PathIO& io, const NeeIO& nee, unsigned long long* ctr) {
    int gb = grid > 0 ? grid : 1;
    if (qcap == 0) gb = std::min(gb, sc.ring_threads / kBlock);  // one ring per resident thread
    dim3 b(kBlock);
    if (qcap != 1 && (!nee.fb_slot || !nee.fb_len)) return hipErrorInvalidValue;  // the fallback list is required
    switch (qcap) {
        case 0: hipLaunchKernelGGL((k_path_nee<0, false>), dim3(resident_grid(k_path_nee<0, false>, gb, grid)), b, 0, st, sc, sp, io, nee, ctr); break;
        case 1: hipLaunchKernelGGL((k_path_nee<1, false>), dim3(resident_grid(k_path_nee<1, false>, gb, grid)), b, 0, st, sc, sp, io, nee, ctr); break;
        case 16: hipLaunchKernelGGL((k_path_nee<16, false>), dim3(resident_grid(k_path_nee<16, false>, gb, grid)), b, 0, st, sc, sp, io, nee, ctr); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// the vertices k_path_nee listed (multi-level octrees only; a resident grid, the list's length read on the device)
hipError_t launch_path_nee_fallback(hipStream_t st, int grid, int qcap, const DevScene& sc, const DevSpectra* sp,
                                    const PathIO& io, const NeeIO& nee, unsigned long long* ctr) {
    int gb = std::min(grid > 0 ? grid : 1, kFallbackBlocks);
    if (qcap == 0) gb = std::min(gb, sc.ring_threads / kBlock);  // one ring per resident thread
    dim3 b(kBlock);
    switch (qcap) {
        case 0: hipLaunchKernelGGL((k_path_nee<0, true>), dim3(resident_grid(k_path_nee<0, true>, gb, grid)), b, 0, st, sc, sp, io, nee, ctr); break;
        case 16: hipLaunchKernelGGL((k_path_nee<16, true>), dim3(resident_grid(k_path_nee<16, true>, gb, grid)), b, 0, st, sc, sp, io, nee, ctr); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_occluded(hipStream_t st, int qcap, const DevScene& sc, int n, const float4* o, const float4* d,
                           int* out, unsigned long long* ctr, bool path) {
    int gb = grid_for(n, 0);
    if (qcap == 0) gb = std::min(gb, sc.ring_threads / kBlock);
    dim3 g(gb > 0 ? gb : 1), b(kBlock);
    if (path && qcap != 1) {
        if (!sc.coop_ok) return hipErrorInvalidValue;
        if (qcap == 0) hipLaunchKernelGGL(k_occluded_path<0>, g, b, 0, st, sc, n, o, d, out, ctr);
        else if (qcap == 16) hipLaunchKernelGGL(k_occluded_path<16>, g, b, 0, st, sc, n, o, d, out, ctr);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    switch (qcap) {
        case 0: hipLaunchKernelGGL(k_occluded<0>, g, b, 0, st, sc, n, o, d, out, ctr); break;
        case 1: hipLaunchKernelGGL(k_occluded<1>, g, b, 0, st, sc, n, o, d, out, ctr); break;
        case 16: hipLaunchKernelGGL(k_occluded<16>, g, b, 0, st, sc, n, o, d, out, ctr); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_path_film(hipStream_t st, int grid, const DevSpectra* sp, const DevFilm& film, const PathFilmIO& io,
                            unsigned long long* ctr) {
    hipLaunchKernelGGL(k_path_film, dim3(resident_grid(k_path_film, grid_for(io.n_pixels, grid), grid)), dim3(kBlock), 0, st, sp, film, io, ctr);
    return hipGetLastError();
}

hipError_t launch_resolve(hipStream_t st, int n, const float4* film, const float* a, const float* b, unsigned char* out,
                          int srgb) {
    hipLaunchKernelGGL(k_resolve, dim3(grid_for(n, 0)), dim3(kBlock), 0, st, n, film, a, b, out, srgb);
    return hipGetLastError();
}

hipError_t launch_film_gather(hipStream_t st, int n, const int* work, const float4* film, float4* out) {
    hipLaunchKernelGGL(k_film_gather, dim3(grid_for(n, 2048)), dim3(kBlock), 0, st, n, work, film, out);
    return hipGetLastError();
}

hipError_t launch_film_scatter(hipStream_t st, int n, const int* work, const float4* in, float4* film) {
    hipLaunchKernelGGL(k_film_scatter, dim3(grid_for(n, 2048)), dim3(kBlock), 0, st, n, work, in, film);
    return hipGetLastError();
}

hipError_t launch_bin_materials(hipStream_t st, int grid, const DevScene& sc, const BinIO& io) {
    hipLaunchKernelGGL(k_bin_materials, dim3(resident_grid(k_bin_materials, grid, grid)), dim3(kBlock), 0, st, sc, io);
    return hipGetLastError();
}


}  // namespace rtmi
