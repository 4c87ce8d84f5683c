// Coherence sort of a path-mode ray queue (multi-level octrees): rays are reordered by (direction octant, 27-bit
// Morton code of the origin within the scene bounds) with a device radix sort, then gathered into a side queue
// that the bounce's trace and shade kernels read.  Traversal results are per ray, so the order changes nothing
// but which rays share a wave: neighbouring rays walk the same nodes and leaves (fewer divergent fetches).
#include <hipcub/hipcub.hpp>

#include "rt_internal.h"

#ifndef RT_SORT_KEY
#define RT_SORT_KEY 4
#endif
#ifndef RT_SORT_DIRB
#define RT_SORT_DIRB 3       // direction: octant + 2 x DIRB bits of the octahedral position
#endif
#ifndef RT_SORT_ORGB
#define RT_SORT_ORGB 7       // origin: ORGB bits per axis (Morton)
#endif

namespace rtmi {
namespace {

constexpr int kKeyBits = RT_SORT_KEY == 4 ? 3 + 2 * RT_SORT_DIRB + 3 * RT_SORT_ORGB : 30;
static_assert(kKeyBits <= 32, "sort key wider than 32 bits");

__device__ __forceinline__ unsigned spread3(unsigned v) {  // 9 bits -> every third bit of 27
    v &= 0x1ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ void __launch_bounds__(kBlockThreads) k_sort_keys(int n, const float4* __restrict__ o,
                                                              const float4* __restrict__ d, float4 lo, float4 scale,
                                                              unsigned* __restrict__ keys, int* __restrict__ vals,
                                                              const int* __restrict__ count) {
    const int nv = count ? *count : n;  // slots past the device count sort last (largest key, stable)
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        if (k >= nv) {
            keys[k] = 0xffffffffu;
            vals[k] = k;
            continue;
        }
        float4 p = o[k], v = d[k];
        auto q = [](float x) {
            x = x < 0.f ? 0.f : (x > 511.f ? 511.f : x);
            return (unsigned)x;
        };
        unsigned m = spread3(q((p.x - lo.x) * scale.x)) << 2 | spread3(q((p.y - lo.y) * scale.y)) << 1 |
                     spread3(q((p.z - lo.z) * scale.z));
        unsigned oct = (v.x < 0.f ? 4u : 0u) | (v.y < 0.f ? 2u : 0u) | (v.z < 0.f ? 1u : 0u);
#if RT_SORT_KEY == 1
        keys[k] = m << 3 | oct;  // origin-major
#elif RT_SORT_KEY == 4
        {  // octant, then the octahedral position on a 2^B x 2^B grid, then an origin Morton code of 3 x ORGB bits
            constexpr int B = RT_SORT_DIRB, OB = RT_SORT_ORGB;
            float s = fabsf(v.x) + fabsf(v.y) + fabsf(v.z);
            const float G = (float)(1 << B);
            unsigned ux = (unsigned)fminf(fabsf(v.x) / s * G, G - 1), uy = (unsigned)fminf(fabsf(v.y) / s * G, G - 1);
            unsigned mo = spread3(q((p.x - lo.x) * scale.x) >> (9 - OB)) << 2 |
                          spread3(q((p.y - lo.y) * scale.y) >> (9 - OB)) << 1 | spread3(q((p.z - lo.z) * scale.z) >> (9 - OB));
            keys[k] = ((oct << (2 * B) | ux << B | uy) << (3 * OB)) | mo;
        }
#else
        keys[k] = oct << 27 | m;  // direction octant first
#endif
        vals[k] = k;
    }
}

__global__ void __launch_bounds__(kBlockThreads) k_sort_gather(int n, const int* __restrict__ perm,
                                                                const float4* __restrict__ o,
                                                                const float4* __restrict__ d,
                                                                const int* __restrict__ slot, float4* __restrict__ so,
                                                                float4* __restrict__ sd, int* __restrict__ ss,
                                                                const int* __restrict__ count) {
    const int nv = count ? *count : n;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < nv; k += gridDim.x * blockDim.x) {
        int j = perm[k];
        so[k] = o[j];
        sd[k] = d[j];
        ss[k] = slot[j];
    }
}

}  // namespace

size_t sort_rays_temp_bytes(int nmax) {
    size_t bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const unsigned*)nullptr, (unsigned*)nullptr,
                                       (const int*)nullptr, (int*)nullptr, nmax, 0, kKeyBits);
    return bytes;
}

hipError_t launch_sort_rays(hipStream_t st, int n, const SortRaysIO& io) {
    if (n <= 0) return hipSuccess;
    int g = (n + kBlockThreads - 1) / kBlockThreads;
    g = g < 8192 ? g : 8192;
    hipLaunchKernelGGL(k_sort_keys, dim3(g), dim3(kBlockThreads), 0, st, n, io.o, io.d, io.lo, io.scale, io.keys,
                       io.vals, io.count);
    size_t bytes = io.temp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(io.temp, bytes, io.keys, io.keys_alt, io.vals, io.vals_alt, n, 0,
                                                      kKeyBits, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sort_gather, dim3(g), dim3(kBlockThreads), 0, st, n, io.vals_alt, io.o, io.d, io.slot, io.so,
                       io.sd, io.ss, io.count);
    return hipGetLastError();
}

}  // namespace rtmi
