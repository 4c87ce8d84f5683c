// Coherence sorts of the multi-level path queues: the bounce rays of a depth by their ray key
// (direction octant, direction cell on an octahedral grid, Morton code of the origin: ray_sort_key, written by the
// shade kernel beside each appended ray) and the deferred NEE vertices by the Morton code of their shading point
// (written by k_path_shade_full).  Traversal results are per ray, so the order changes nothing but which rays share a
// wave: neighbouring rays walk the same nodes and leaves.
//
// A hand-written stable LSD radix sort that runs entirely on the device (no host read of the queue length):
//   k_rs_prep     the queue's shard lengths -> n and the shard prefix (meta), read by every later kernel;
//   per pass of one digit (RB bits: 9 for the 18-bit ray key, 8 for the 24-bit NEE key):
//   k_rs_hist     block b counts the digits of its chunk of the (concatenated) queue in LDS;
//   k_rs_offsets  block = digit: the exclusive scan of the digit's counts over the blocks and the digit's total;
//   k_rs_scatter  block b scans the digit totals into digit starts, then walks its chunk in tiles of kRsIpt items per
//                 thread, ranked in order (stable) in sub-tiles of one item per thread: a wave ranks its items among
//                 the same digit with nbits ballots (lane order), the sub-tile's waves are prefixed per digit through
//                 LDS, and a running count per digit (one digit per thread) carries the order across sub-tiles; the
//                 tile is then staged in LDS in digit order and stored in runs of consecutive addresses.  The
//                 first pass reads the keys at the queue positions; the last one writes the queue positions (rays:
//                 the trace kernel gathers them, TraceIO perm) or the NEE slots (in place) in the sorted queue's
//                 sharded layout, the sorted order split evenly over the shards.
// Stability matters: within a key, rays keep their slot order, so the shade kernel's per-slot state reads stay
// close (an unstable atomic counting sort with the same keys measured CFG3 463 -> 375 Msamples/s in round 2).
#include <algorithm>

#include "rt_internal.h"

namespace rtmi {
namespace {

// Digit width per sort (RB bits: 1 << RB digits, one per thread of a 1 << RB-thread block, tiles of 1 << RB items):
// the 18-bit ray key sorts in 2 passes of 9 bits (r03 A/B: CFG3 +0.6 % over 3 passes of 6), the 24-bit NEE key in 3
// passes of 8 (with 9-bit digits its passes cost more: CFG4 -0.7 %).
#ifndef RT_RS_RAY_BITS
#define RT_RS_RAY_BITS 9
#endif
#ifndef RT_RS_NEE_BITS
#define RT_RS_NEE_BITS 8
#endif
constexpr int kRsGrid = 1024;  // blocks of the histogram / scatter kernels (4 per CU)
// items per thread of a scatter tile (tiles of kRsIpt x 2^RB items); r04 A/B against round 3's tiles of one item per
// thread with scattered stores: the same time (CFG3 1.93 vs 2.03 ms, CFG4 5.11 vs 5.08 ms of sort per step), fewer
// bytes written
constexpr int kRsIpt = 8;
constexpr int kRsBinsMax = 512;

// meta: [0] n, [1 .. kShards + 1] the exclusive prefix of the shard lengths
__global__ void k_rs_prep(const int* __restrict__ len, int* __restrict__ meta) {
    if (threadIdx.x == 0) {
        int p = 0;
        for (int j = 0; j < kShards; ++j) {
            meta[1 + j] = p;
            p += len[j * kQStride];
        }
        meta[1 + kShards] = p;
        meta[0] = p;
    }
}

template <int kRsTile>
__device__ __forceinline__ int rs_chunk(int n) {  // items per block: a multiple of the tile
    const int c = (n + kRsGrid - 1) / kRsGrid;
    return (c + kRsTile - 1) / kRsTile * kRsTile;
}
// queue position of concatenated item k (shards in order)
__device__ __forceinline__ int rs_pos(const int* meta, int S, int k) {
    int j = 0;
#pragma unroll
    for (int u = 1; u < kShards; ++u) j += k >= meta[1 + u] ? 1 : 0;
    int base = meta[1];
#pragma unroll
    for (int u = 1; u < kShards; ++u) base = j == u ? meta[1 + u] : base;
    return j * S + (k - base);
}

enum { SRC_ARRAY = 0, SRC_RAYQ = 1, SRC_NEEQ = 2 };       // where a pass reads (key, value)
enum { DST_ARRAY = 0, DST_PERM = 1, DST_NEEQ = 2 };       // where it writes them

struct RsPass {
    const int* meta;
    int S;                       // the queue's shard stride
    // sources: SRC_ARRAY keys_in / vals_in[k]; SRC_RAYQ qkey[pos], value pos; SRC_NEEQ qkey[pos], value slot[pos]
    const unsigned* keys_in; const int* vals_in;
    const unsigned* qkey; const int* qslot;
    int shift, nbits;
    int* hist;                   // kRsBins x kRsGrid (digit-major): counts, then (k_rs_offsets) each block's
                                 // exclusive start within its digit
    int* tot;                    // kRsBins digit totals (k_rs_offsets)
    // destinations: DST_ARRAY keys_out / vals_out[k']; DST_PERM the values (queue positions) in the sorted queue's
    // sharded layout (perm: the trace kernel gathers the rays); DST_NEEQ the NEE queue's slots in place; both rewrite
    // the shard lengths `len`
    unsigned* keys_out; int* vals_out;
    int* nslot;
    int* len;
};

template <int SRC>
__device__ __forceinline__ void rs_load(const RsPass& p, int k, unsigned& key, int& val) {
    if constexpr (SRC == SRC_ARRAY) {
        key = p.keys_in[k];
        val = p.vals_in[k];
    } else {
        const int pos = rs_pos(p.meta, p.S, k);
        key = p.qkey[pos];
        val = SRC == SRC_RAYQ ? pos : p.qslot[pos];
    }
}

// barrier for LDS hand-offs only: waits for the block's LDS operations, not for its global loads in flight
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int SRC, int RB>
__global__ void __launch_bounds__(1 << RB) k_rs_hist(RsPass p) {
    constexpr int kRsBins = 1 << RB, kRsThreads = kRsBins;
    constexpr int U = 4;  // items in flight per thread
    __shared__ int h[kRsBins];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int n = p.meta[0], c = rs_chunk<kRsIpt * kRsThreads>(n);  // (the scatter kernel's chunks)
    const int b0 = (int)blockIdx.x * c, b1 = min(b0 + c, n);
    const unsigned mask = (1u << p.nbits) - 1u;
    for (int k0 = b0 + (int)threadIdx.x; k0 < b1; k0 += U * kRsThreads) {
        unsigned key[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = k0 + u * kRsThreads;
            int val;
            key[u] = 0;
            if (k < b1) rs_load<SRC>(p, k, key[u], val);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + u * kRsThreads < b1) atomicAdd(&h[(key[u] >> p.shift) & mask], 1);
    }
    __syncthreads();
    p.hist[threadIdx.x * kRsGrid + blockIdx.x] = h[threadIdx.x];  // digit-major: k_rs_offsets scans a digit's row
}

// block d = digit d, thread b = block b of the histogram kernel: the exclusive scan of row d over the blocks (in
// place), and the digit's total in tot[d] (the scatter kernel turns the totals into digit starts)
__global__ void __launch_bounds__(kRsGrid) k_rs_offsets(int* __restrict__ hist, int* __restrict__ tot) {
    __shared__ int wsum[kRsGrid / 64];
    int* row = hist + (size_t)blockIdx.x * kRsGrid;
    const int b = threadIdx.x, lane = b & 63, w = b >> 6;
    const int v = row[b];
    int x = v;  // inclusive wave scan
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        x += lane >= off ? y : 0;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int i = 0; i < kRsGrid / 64; ++i) base += i < w ? wsum[i] : 0;
    row[b] = base + x - v;
    if (b == kRsGrid - 1) tot[blockIdx.x] = base + x;
}

__device__ __forceinline__ int rs_lane() {
    return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Tiles of kRsIpt items per thread (kRsIpt x 2^RB items), ranked in kRsIpt sub-tiles of one item per thread, in
// order (stable): a wave ranks its items among equal digits with nbits ballots, the sub-tile's waves are prefixed
// per digit through LDS, and a running count per digit (one digit per thread) carries the order across sub-tiles and
// tiles.  Within a tile the items of one digit get consecutive destinations, so the tile is staged in LDS in digit
// order and written back from there: consecutive threads store consecutive addresses (runs of kRsIpt items per digit
// on average) instead of one scattered 4-B store per item (r03: 2.7x the algorithmic bytes written).
template <int SRC, int DST, int RB>
__global__ void __launch_bounds__(1 << RB) k_rs_scatter(RsPass p) {
    constexpr int kRsBins = 1 << RB, kRsThreads = kRsBins, kRsTile = kRsIpt * kRsThreads;
    constexpr int NW = kRsThreads / 64;
    __shared__ int wcnt[NW][kRsBins];
    __shared__ int wpre[NW][kRsBins];
    __shared__ unsigned skey[kRsTile];
    __shared__ int sval[kRsTile];
    __shared__ int dstart[kRsBins];  // tile-local start of digit d (the tile in digit order)
    __shared__ int rstart[kRsBins];  // destination of digit d's first item of the tile
    __shared__ int wsum[NW];
    const int n = p.meta[0], c = rs_chunk<kRsTile>(n);
    const int b0 = (int)blockIdx.x * c, b1 = min(b0 + c, n);
    if (b0 >= b1 && blockIdx.x != 0) return;  // (no items: a deep bounce's few rays leave most blocks idle; block 0
                                              // always rewrites the shard lengths)
    const int tid = threadIdx.x, w = tid >> 6, lane = rs_lane();
    const unsigned mask = (1u << p.nbits) - 1u;
    {  // the digits' starts: exclusive scan of the digit totals (Hillis-Steele over the kRsBins digits, in wpre[0])
        int* sc = wpre[0];
        sc[tid] = p.tot[tid];
        __syncthreads();
        for (int off = 1; off < kRsBins; off <<= 1) {
            const int y = tid >= off ? sc[tid - off] : 0;
            __syncthreads();
            sc[tid] += y;
            __syncthreads();
        }
    }
    // this thread's digit (tid): next output index
    int run = wpre[0][tid] - p.tot[tid] + p.hist[tid * kRsGrid + blockIdx.x];
    __syncthreads();
    const int S2 = shard_stride(n, kShards);      // the sorted queue: item k' at shard k' / S2
    if (DST != DST_ARRAY && blockIdx.x == 0 && tid < kShards) {
        const int cc = n - tid * S2;
        p.len[tid * kQStride] = cc < 0 ? 0 : (cc > S2 ? S2 : cc);
    }
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int t0 = b0; t0 < b1; t0 += kRsTile) {  // (block-uniform trip count)
        unsigned key[kRsIpt];
        int val[kRsIpt], dst[kRsIpt];
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j) {  // all of the tile's loads in flight at once
            const int k = t0 + j * kRsThreads + tid;
            key[j] = 0;
            val[j] = 0;
            if (k < b1) rs_load<SRC>(p, k, key[j], val[j]);
        }
        const int run0 = run;
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j) {
            const bool valid = t0 + j * kRsThreads + tid < b1;
            const unsigned dg = (key[j] >> p.shift) & mask;
            // lanes of this wave with the same digit: AND over the digit's bits of (ballot of the bit, or its complement)
            uint64_t m = __ballot(valid);
            for (int bit = 0; bit < p.nbits; ++bit) {
                const uint64_t bb = __ballot((dg >> bit) & 1u);
                m &= ((dg >> bit) & 1u) ? bb : ~bb;
            }
            const int rank = __popcll(m & lt);
#pragma unroll
            for (int i = 0; i < NW; ++i) wcnt[i][tid] = 0;
            lds_barrier();
            if (valid && rank == 0) wcnt[w][dg] = __popcll(m);  // the digit's lowest lane reports the wave's count
            lds_barrier();
            {  // digit tid: prefix over the sub-tile's waves, then carry the running count
                int r = run;
#pragma unroll
                for (int i = 0; i < NW; ++i) {
                    wpre[i][tid] = r;
                    r += wcnt[i][tid];
                }
                run = r;
            }
            lds_barrier();
            dst[j] = valid ? wpre[w][dg] + rank : -1;
        }
        // digit tid's items of this tile: destinations [run0, run); its tile-local start = the exclusive scan of the
        // tile's digit counts
        const int cnt = run - run0;
        int x = cnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(x, off);
            x += lane >= off ? y : 0;
        }
        if (lane == 63) wsum[w] = x;
        lds_barrier();
        int base = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) base += i < w ? wsum[i] : 0;
        dstart[tid] = base + x - cnt;
        rstart[tid] = run0;
        lds_barrier();
#pragma unroll
        for (int j = 0; j < kRsIpt; ++j)
            if (dst[j] >= 0) {
                const unsigned dg = (key[j] >> p.shift) & mask;
                const int l = dstart[dg] + (dst[j] - rstart[dg]);
                skey[l] = key[j];
                sval[l] = val[j];
            }
        lds_barrier();
        const int tn = min(kRsTile, b1 - t0);
        for (int l = tid; l < tn; l += kRsThreads) {  // in digit order: consecutive threads, consecutive addresses
            const unsigned kk = skey[l];
            const unsigned dg = (kk >> p.shift) & mask;
            const int d = rstart[dg] + (l - dstart[dg]);
            if constexpr (DST == DST_ARRAY) {
                p.keys_out[d] = kk;
                p.vals_out[d] = sval[l];
            } else {
                p.nslot[(d / S2) * p.S + d % S2] = sval[l];
            }
        }
        lds_barrier();  // (skey / sval / dstart / rstart are rewritten by the next tile)
    }
}

template <int SRC, int DST, int RB>
void rs_launch(hipStream_t st, const RsPass& p) {
    hipLaunchKernelGGL((k_rs_hist<SRC, RB>), dim3(kRsGrid), dim3(1 << RB), 0, st, p);
    hipLaunchKernelGGL(k_rs_offsets, dim3(1 << RB), dim3(kRsGrid), 0, st, p.hist, p.tot);
    hipLaunchKernelGGL((k_rs_scatter<SRC, DST, RB>), dim3(kRsGrid), dim3(1 << RB), 0, st, p);
}

// the passes of a `bits`-bit key, <= RB bits each (split evenly), ping-ponging between the two arrays
template <int SRC, int DST, int RB>
hipError_t rs_sort(hipStream_t st, int bits, RsPass p, unsigned* ka, unsigned* kb, int* va, int* vb) {
    static_assert(RB >= 6 && (1 << RB) <= kRsBinsMax, "digit width");
    // (the NEE queue is sorted in place: its first pass must finish reading the slots before any is rewritten)
    const int passes = std::max((bits + RB - 1) / RB, DST == DST_NEEQ ? 2 : 1);
    const int per = (bits + passes - 1) / passes;
    hipLaunchKernelGGL(k_rs_prep, dim3(1), dim3(64), 0, st, p.len, const_cast<int*>(p.meta));
    for (int i = 0; i < passes; ++i) {
        p.shift = i * per;
        p.nbits = bits - p.shift < per ? bits - p.shift : per;
        const bool first = i == 0, last = i == passes - 1;
        p.keys_out = (i & 1) ? kb : ka;
        p.vals_out = (i & 1) ? vb : va;
        if (first && last) rs_launch<SRC, DST, RB>(st, p);
        else if (first) rs_launch<SRC, DST_ARRAY, RB>(st, p);
        else if (last) rs_launch<SRC_ARRAY, DST, RB>(st, p);
        else rs_launch<SRC_ARRAY, DST_ARRAY, RB>(st, p);
        p.keys_in = p.keys_out;
        p.vals_in = p.vals_out;
    }
    return hipGetLastError();
}

}  // namespace

size_t sort_temp_bytes() { return sizeof(int) * ((size_t)kRsGrid * kRsBinsMax + kRsBinsMax + 64); }

hipError_t launch_sort_rays(hipStream_t st, const SortRaysIO& io) {
    RsPass p{};
    int* hist = static_cast<int*>(io.temp);
    p.hist = hist;
    p.tot = hist + (size_t)kRsGrid * kRsBinsMax;
    p.meta = p.tot + kRsBinsMax;
    p.S = io.S;
    p.qkey = io.qkey;
    p.nslot = io.perm;
    p.len = io.len;
    const int bits = 3 + 2 * io.dir_bits + 3 * io.org_bits;
    return rs_sort<SRC_RAYQ, DST_PERM, RT_RS_RAY_BITS>(st, bits, p, io.keys, io.keys_alt, io.vals, io.vals_alt);
}

hipError_t launch_sort_nee(hipStream_t st, const SortNeeIO& io) {
    RsPass p{};
    int* hist = static_cast<int*>(io.temp);
    p.hist = hist;
    p.tot = hist + (size_t)kRsGrid * kRsBinsMax;
    p.meta = p.tot + kRsBinsMax;
    p.S = io.S;
    p.qkey = io.key;
    p.qslot = io.slot;
    p.nslot = io.slot;  // in place: the first pass copied the slots into the values
    p.len = io.len;
    return rs_sort<SRC_NEEQ, DST_NEEQ, RT_RS_NEE_BITS>(st, 3 * io.org_bits, p, io.keys, io.keys_alt, io.vals, io.vals_alt);
}

}  // namespace rtmi
