// Coherence sort of a path-mode ray queue (multi-level octrees): rays are reordered by (direction octant, direction
// cell on an octahedral grid, Morton code of the origin within the scene bounds) with a stable device radix sort,
// then gathered into a side queue that the bounce's trace and shade kernels read.  Traversal results are per ray, so
// the order changes nothing but which rays share a wave: neighbouring rays walk the same nodes and leaves.  The sort
// must be stable: within a key, rays keep their slot order, so the shade kernel's per-slot state reads stay close
// (an atomic counting sort with the same keys, unstable, measured CFG3 463 -> 375 Msamples/s).
#include <hipcub/hipcub.hpp>

#include "rt_internal.h"

namespace rtmi {
namespace {


__device__ __forceinline__ unsigned spread3(unsigned v) {  // 9 bits -> every third bit of 27
    v &= 0x1ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

// (both queues hold interleaved (o, d) pairs: ray k at o[2k], d[2k] with d = o + 1, one 32-B line per ray)
// key = direction octant, then the octahedral position of the direction on a 2^B x 2^B grid, then a Morton code of
// the origin with O bits per axis (DESIGN.md §6 key table).  Entry k of the sort is the k-th live ray of the sharded
// queue (shards in order); its value is the ray's queue position.
__global__ void __launch_bounds__(kBlockThreads) k_sort_keys(int n, const int* __restrict__ len, int S,
                                                              const float4* __restrict__ o,
                                                              const float4* __restrict__ d, float4 lo, float4 scale,
                                                              int kDirB, int kOrgB, int org_major,
                                                              unsigned* __restrict__ keys, int* __restrict__ vals) {
    int pre[kShards + 1];
    pre[0] = 0;
#pragma unroll
    for (int j = 0; j < kShards; ++j) pre[j + 1] = pre[j] + len[j * kQStride];
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        int j = 0;
#pragma unroll
        for (int u = 1; u < kShards; ++u) j += k >= pre[u] ? 1 : 0;
        int base = pre[0];
#pragma unroll
        for (int u = 1; u < kShards; ++u) base = j == u ? pre[u] : base;
        const int pos = j * S + (k - base);
        float4 p = o[2 * pos], v = d[2 * pos];
        auto q = [](float x) {
            x = x < 0.f ? 0.f : (x > 511.f ? 511.f : x);
            return (unsigned)x;
        };
        unsigned oct = (v.x < 0.f ? 4u : 0u) | (v.y < 0.f ? 2u : 0u) | (v.z < 0.f ? 1u : 0u);
        float sum = fabsf(v.x) + fabsf(v.y) + fabsf(v.z);
        const float G = (float)(1 << kDirB);
        unsigned ux = (unsigned)fminf(fabsf(v.x) / sum * G, G - 1), uy = (unsigned)fminf(fabsf(v.y) / sum * G, G - 1);
        unsigned mo = spread3(q((p.x - lo.x) * scale.x) >> (9 - kOrgB)) << 2 |
                      spread3(q((p.y - lo.y) * scale.y) >> (9 - kOrgB)) << 1 |
                      spread3(q((p.z - lo.z) * scale.z) >> (9 - kOrgB));
        const unsigned dk = oct << (2 * kDirB) | ux << kDirB | uy;
        keys[k] = org_major ? (mo << (3 + 2 * kDirB)) | dk : (dk << (3 * kOrgB)) | mo;
        vals[k] = pos;
    }
}

// sorted entry k -> shard k / S2 of the side queue (S2 = shard_stride(n, kShards) <= S; sorted queues have kShards: the sorted order split evenly over
// the shards), and the side queue's shard lengths replace the queue's (every reader of this bounce uses the side
// queue)
__global__ void __launch_bounds__(kBlockThreads) k_sort_gather(int n, const int* __restrict__ perm, int S, int S2,
                                                                const float4* __restrict__ o,
                                                                const float4* __restrict__ d,
                                                                float4* __restrict__ so,
                                                                float4* __restrict__ sd, int* __restrict__ ss,
                                                                int* __restrict__ len) {
    if (blockIdx.x == 0 && threadIdx.x < kShards) {
        const int c = n - (int)threadIdx.x * S2;
        len[threadIdx.x * kQStride] = c < 0 ? 0 : (c > S2 ? S2 : c);
    }
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const int j = perm[k];
        const int pos = (k / S2) * S + k % S2;
        const float4 oj = o[2 * j];
        so[2 * pos] = oj;
        sd[2 * pos] = d[2 * j];
        ss[pos] = __float_as_int(oj.w);  // bounce rays carry their slot in o.w: two scattered reads per ray, not three
    }
}

// NEE queue coherence sort (mixed scenes, RTMI_SORT_NEE): the deferred NEE vertices of one bounce reordered by the
// Morton code of their shading point (org_bits per axis; k_path_shade_full writes it beside the queue entry), so the
// shadow rays of a wave start close together and walk the same BVH nodes toward each light.  k_path_nee still traces and adds a vertex's lights in light order, and the
// vertices are independent of each other (one slot each), so the film is unchanged.  Entry k is the k-th queued
// vertex (shards in order); its value is the vertex's slot.
__global__ void __launch_bounds__(kBlockThreads) k_nee_keys(int n, const int* __restrict__ len, int S,
                                                             const int* __restrict__ slot,
                                                             const unsigned* __restrict__ key,
                                                             unsigned* __restrict__ keys, int* __restrict__ vals) {
    int pre[kShards + 1];
    pre[0] = 0;
#pragma unroll
    for (int j = 0; j < kShards; ++j) pre[j + 1] = pre[j] + len[j * kQStride];
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        int j = 0;
#pragma unroll
        for (int u = 1; u < kShards; ++u) j += k >= pre[u] ? 1 : 0;
        int base = pre[0];
#pragma unroll
        for (int u = 1; u < kShards; ++u) base = j == u ? pre[u] : base;
        const int pos = j * S + (k - base);
        keys[k] = key[pos];
        vals[k] = slot[pos];
    }
}

// sorted entry k -> shard k / S2 of the NEE queue (in place: the slots were copied into the sort's values), and the
// shard lengths rewritten for that split
__global__ void __launch_bounds__(kBlockThreads) k_nee_scatter(int n, const int* __restrict__ sorted, int S, int S2,
                                                                int* __restrict__ slot, int* __restrict__ len) {
    if (blockIdx.x == 0 && threadIdx.x < kShards) {
        const int c = n - (int)threadIdx.x * S2;
        len[threadIdx.x * kQStride] = c < 0 ? 0 : (c > S2 ? S2 : c);
    }
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
        slot[(k / S2) * S + k % S2] = sorted[k];
}

}  // namespace

size_t sort_rays_temp_bytes(int nmax) {
    size_t bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const unsigned*)nullptr, (unsigned*)nullptr,
                                       (const int*)nullptr, (int*)nullptr, nmax, 0, 32);
    return bytes;
}

hipError_t launch_sort_rays(hipStream_t st, int n, const SortRaysIO& io) {
    if (n <= 0) return hipSuccess;
    int g = (n + kBlockThreads - 1) / kBlockThreads;
    g = g < 8192 ? g : 8192;
    const int key_bits = 3 + 2 * io.dir_bits + 3 * io.org_bits;
    hipLaunchKernelGGL(k_sort_keys, dim3(g), dim3(kBlockThreads), 0, st, n, io.len, io.S, io.o, io.d, io.lo, io.scale,
                       io.dir_bits, io.org_bits, io.org_major, io.keys, io.vals);
    size_t bytes = io.temp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(io.temp, bytes, io.keys, io.keys_alt, io.vals, io.vals_alt, n, 0,
                                                      key_bits, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sort_gather, dim3(g), dim3(kBlockThreads), 0, st, n, io.vals_alt, io.S, shard_stride(n, kShards),
                       io.o, io.d, io.so, io.sd, io.ss, io.len);
    return hipGetLastError();
}

hipError_t launch_sort_nee(hipStream_t st, int n, const SortNeeIO& io) {
    if (n <= 0) return hipSuccess;
    int g = (n + kBlockThreads - 1) / kBlockThreads;
    g = g < 8192 ? g : 8192;
    hipLaunchKernelGGL(k_nee_keys, dim3(g), dim3(kBlockThreads), 0, st, n, io.len, io.S, io.slot, io.key, io.keys,
                       io.vals);
    size_t bytes = io.temp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(io.temp, bytes, io.keys, io.keys_alt, io.vals, io.vals_alt, n, 0,
                                                      3 * io.org_bits, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_nee_scatter, dim3(g), dim3(kBlockThreads), 0, st, n, io.vals_alt, io.S,
                       shard_stride(n, kShards), io.slot, io.len);
    return hipGetLastError();
}

}  // namespace rtmi
