// FETCH_SIZE / WRITE_SIZE calibration for the access shapes of the path tracer's kernels (MI355X_MICROARCH §HBM:
// the counters are validated only for wide coalesced streams).  Each kernel moves a known number of bytes over a
// 1 GiB buffer (beyond the 256 MiB Infinity Cache), one launch each; rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE)
// per launch divided by the bytes printed here gives the factor per shape:
//   coalesced16   every lane reads one float4, consecutive lanes consecutive addresses (the ray / state streams)
//   gather32      every lane reads 32 B (two float4) at a random 32-B aligned record (the sorted-ray gather)
//   gather16      every lane reads one float4 at a random 16-B aligned address (scattered slot fields)
//   gather128     every lane reads one 128-B record (8 float4) at a random record (the BVH node lines)
//   store16       every lane writes one float4, coalesced
//   scatter32     every lane writes 32 B at a random 32-B record
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/_build/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d out -o pmc --output-format csv -- tools/_build/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                     \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// n_items work items; each kernel writes one float per item to sink (so no load is dead)
__global__ void k_coalesced16(const float4* __restrict__ a, int n, float* sink) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { float4 v = a[i]; sink[i] = v.x + v.y + v.z + v.w; }
}
__global__ void k_gather(const float4* __restrict__ a, int n, uint32_t nrec, int f4_per_rec, float* sink) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = hash32((uint32_t)i * 2654435761u + 12345u) % nrec;
    const float4* p = a + (size_t)r * f4_per_rec;
    float s = 0.f;
    for (int k = 0; k < f4_per_rec; ++k) { float4 v = p[k]; s += v.x + v.y + v.z + v.w; }
    sink[i] = s;
}
__global__ void k_store16(float4* __restrict__ a, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}
__global__ void k_scatter32(float4* __restrict__ a, int n, uint32_t nrec) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = hash32((uint32_t)i * 2654435761u + 777u) % nrec;
    a[2 * (size_t)r] = make_float4((float)i, 1.f, 2.f, 3.f);
    a[2 * (size_t)r + 1] = make_float4(4.f, 5.f, 6.f, 7.f);
}

int main() {
    const size_t bytes = (size_t)1 << 30;  // 1 GiB: beyond the Infinity Cache
    const size_t nf4 = bytes / 16;
    float4 *a = nullptr, *b = nullptr;
    float* sink = nullptr;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    const int n = 16 << 20;  // 16 Mi work items per launch
    CHK(hipMalloc(&sink, (size_t)n * sizeof(float)));
    CHK(hipMemset(a, 0, bytes));
    CHK(hipMemset(b, 0, bytes));
    CHK(hipDeviceSynchronize());
    const dim3 blk(256), grd((n + 255) / 256);
    // sink writes are 4 B per item, coalesced (subtract them from WRITE_SIZE of the read kernels)
    hipLaunchKernelGGL(k_coalesced16, grd, blk, 0, 0, a, n, sink);
    std::printf("coalesced16 read_bytes %zu sink_bytes %zu\n", (size_t)n * 16, (size_t)n * 4);
    hipLaunchKernelGGL(k_gather, grd, blk, 0, 0, a, n, (uint32_t)(bytes / 32), 2, sink);
    std::printf("gather32 read_bytes %zu sink_bytes %zu\n", (size_t)n * 32, (size_t)n * 4);
    hipLaunchKernelGGL(k_gather, grd, blk, 0, 0, a, n, (uint32_t)nf4, 1, sink);
    std::printf("gather16 read_bytes %zu sink_bytes %zu\n", (size_t)n * 16, (size_t)n * 4);
    hipLaunchKernelGGL(k_gather, dim3((n / 4 + 255) / 256), blk, 0, 0, a, n / 4, (uint32_t)(bytes / 128), 8, sink);
    std::printf("gather128 read_bytes %zu sink_bytes %zu\n", (size_t)n / 4 * 128, (size_t)n / 4 * 4);
    hipLaunchKernelGGL(k_store16, grd, blk, 0, 0, b, n);
    std::printf("store16 write_bytes %zu\n", (size_t)n * 16);
    hipLaunchKernelGGL(k_scatter32, grd, blk, 0, 0, b, n, (uint32_t)(bytes / 32));
    std::printf("scatter32 write_bytes %zu\n", (size_t)n * 32);
    CHK(hipDeviceSynchronize());
    CHK(hipFree(a));
    CHK(hipFree(b));
    CHK(hipFree(sink));
    return 0;
}
