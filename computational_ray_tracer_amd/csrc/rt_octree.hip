// On-device octree build: the reference inserts triangles one by one (Octtree_Model.h:33-63
// CreateOcttree, 180-277 AddTriangle, 279-358 Split), so its tree depends on insertion order.  The sequential
// process is equivalent to a top-down, level-synchronous one:
//   - a node's arrival sequence A_N is its parent's, filtered by the Möller overlap with N's box, in insertion
//     order (triangles present at the split are routed, later ones forwarded, both in order);
//   - a leaf attempts a split after every append that leaves it with >= capacity triangles, except that a child
//     does not attempt one at creation: attempts happen at sizes k >= max(capacity, s0 + 1), s0 = the triangles
//     it received from its parent's split;
//   - an attempt at size k aborts iff some child box overlaps all of A_N[0..k), so with m_c the first index of
//     A_N not overlapping child c, it succeeds for the first k > max_c m_c.
// These kernels do the per-level work: classify (8 overlap bits per (node, triangle), m_c, child counts) and an
// order-preserving scatter into the children's sequences.  The host (rt_host.cpp, octree_build_device) decides
// splits, lays out the next level and finally renumbers the nodes in the reference's split order.
#include "rt_internal.h"

namespace rtmi {
namespace {

struct B3 {
    float x, y, z;
};
__device__ __forceinline__ B3 bsub(B3 a, B3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ B3 bcross(B3 a, B3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
__device__ __forceinline__ float bdot(B3 a, B3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ float bget(B3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

__device__ __forceinline__ bool axis_ok(float pa, float pb, float rad) {
    float mn, mx;
    if (pa < pb) { mn = pa; mx = pb; } else { mn = pb; mx = pa; }
    return !(mn > rad || mx < -rad);
}
__device__ __forceinline__ bool axis_ok_z12(float p1, float p2, float rad) {
    float mn, mx;
    if (p2 < p1) { mn = p2; mx = p1; } else { mn = p1; mx = p2; }
    return !(mn > rad || mx < -rad);
}
// AABB_triangle_Moller.h:229-474 triBoxOverlap, with the reference's AXISTEST_Z0 that never rejects (:342); the same
// operations in the same order as the host builder's tri_box_overlap
__device__ bool tri_box_overlap(B3 c, B3 h, B3 t0, B3 t1, B3 t2) {
    B3 v0 = bsub(t0, c), v1 = bsub(t1, c), v2 = bsub(t2, c);
    B3 e0 = bsub(v1, v0), e1 = bsub(v2, v1), e2 = bsub(v0, v2);
    float fex, fey, fez;
    fex = fabsf(e0.x); fey = fabsf(e0.y); fez = fabsf(e0.z);
    if (!axis_ok(e0.z * v0.y - e0.y * v0.z, e0.z * v2.y - e0.y * v2.z, fez * h.y + fey * h.z)) return false;
    if (!axis_ok(-e0.z * v0.x + e0.x * v0.z, -e0.z * v2.x + e0.x * v2.z, fez * h.x + fex * h.z)) return false;
    if (!axis_ok_z12(e0.y * v1.x - e0.x * v1.y, e0.y * v2.x - e0.x * v2.y, fey * h.x + fex * h.y)) return false;
    fex = fabsf(e1.x); fey = fabsf(e1.y); fez = fabsf(e1.z);
    if (!axis_ok(e1.z * v0.y - e1.y * v0.z, e1.z * v2.y - e1.y * v2.z, fez * h.y + fey * h.z)) return false;
    if (!axis_ok(-e1.z * v0.x + e1.x * v0.z, -e1.z * v2.x + e1.x * v2.z, fez * h.x + fex * h.z)) return false;
    fex = fabsf(e2.x); fey = fabsf(e2.y); fez = fabsf(e2.z);
    if (!axis_ok(e2.z * v0.y - e2.y * v0.z, e2.z * v1.y - e2.y * v1.z, fez * h.y + fey * h.z)) return false;
    if (!axis_ok(-e2.z * v0.x + e2.x * v0.z, -e2.z * v1.x + e2.x * v1.z, fez * h.x + fex * h.z)) return false;
    if (!axis_ok_z12(e2.y * v1.x - e2.x * v1.y, e2.y * v2.x - e2.x * v2.y, fey * h.x + fex * h.y)) return false;
    float mn, mx;
    auto mm = [&](float a, float b, float cc) {
        mn = mx = a;
        if (b < mn) mn = b;
        if (b > mx) mx = b;
        if (cc < mn) mn = cc;
        if (cc > mx) mx = cc;
    };
    mm(v0.x, v1.x, v2.x);
    if (mn > h.x || mx < -h.x) return false;
    mm(v0.y, v1.y, v2.y);
    if (mn > h.y || mx < -h.y) return false;
    mm(v0.z, v1.z, v2.z);
    if (mn > h.z || mx < -h.z) return false;
    B3 nrm = bcross(e0, e1);  // planeBoxOverlap
    float vmin[3], vmax[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        float v = bget(v0, q), nq = bget(nrm, q), mb = bget(h, q);
        if (nq > 0.0f) { vmin[q] = -mb - v; vmax[q] = mb - v; }
        else { vmin[q] = mb - v; vmax[q] = -mb - v; }
    }
    if (bdot(nrm, {vmin[0], vmin[1], vmin[2]}) > 0.0f) return false;
    if (bdot(nrm, {vmax[0], vmax[1], vmax[2]}) >= 0.0f) return true;
    return false;
}

// One block per node (grid-stride over nodes): the 8 overlap bits of every triangle of the node's sequence against
// its 8 child boxes (cbox: 8 x (mn.xyz, mx.xyz)), then m_c (first index without bit c; len if none) and the
// per-child counts.  stats[9 n] = {max_c m_c, count_0..7}.
__global__ void __launch_bounds__(kBlockThreads) k_oct_classify(int nnodes, const float* __restrict__ cbox,
                                                                 const int* __restrict__ seg,
                                                                 const int* __restrict__ ent,
                                                                 const float* __restrict__ tri9,
                                                                 unsigned char* __restrict__ mask,
                                                                 int* __restrict__ stats) {
    __shared__ float box[48];
    __shared__ int first_miss[8], count[8];
    for (int nd = blockIdx.x; nd < nnodes; nd += gridDim.x) {
        const int b = seg[2 * nd], len = seg[2 * nd + 1];
        if (threadIdx.x < 48) box[threadIdx.x] = cbox[48 * nd + threadIdx.x];
        if (threadIdx.x < 8) { first_miss[threadIdx.x] = len; count[threadIdx.x] = 0; }
        __syncthreads();
        int cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int fm[8] = {len, len, len, len, len, len, len, len};  // this thread's first miss per child (i ascends)
        for (int i = threadIdx.x; i < len; i += blockDim.x) {
            const int t = ent[b + i];
            const float* p = tri9 + 9 * (size_t)t;
            B3 t0 = {p[0], p[1], p[2]}, t1 = {p[3], p[4], p[5]}, t2 = {p[6], p[7], p[8]};
            unsigned m = 0;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float* q = box + 6 * c;
                // OctBuild::overlap: half = (mx - mn) / 2, centre = mn + half
                B3 half = {(q[3] - q[0]) / 2.0f, (q[4] - q[1]) / 2.0f, (q[5] - q[2]) / 2.0f};
                B3 cen = {q[0] + half.x, q[1] + half.y, q[2] + half.z};
                if (tri_box_overlap(cen, half, t0, t1, t2)) { m |= 1u << c; ++cnt[c]; }
                else if (fm[c] == len) fm[c] = i;
            }
            mask[b + i] = (unsigned char)m;
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if (cnt[c]) atomicAdd(&count[c], cnt[c]);
            if (fm[c] < len) atomicMin(&first_miss[c], fm[c]);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int M = 0;
            for (int c = 0; c < 8; ++c) M = first_miss[c] > M ? first_miss[c] : M;
            stats[9 * nd] = M;
            for (int c = 0; c < 8; ++c) stats[9 * nd + 1 + c] = count[c];
        }
        __syncthreads();
    }
}

// One block per splitting node: its sequence scattered, in order, into the children's sequences
// (job[12 j] = {begin, len, k_split, dst_0..dst_7, unused}); s0[8 j + c] = entries of child c that come from
// A_N[0..k_split) (the triangles present when the split happened).  nchild = 1 for the root filter pass.
__global__ void __launch_bounds__(kBlockThreads) k_oct_scatter(int njobs, int nchild, const int* __restrict__ job,
                                                                const int* __restrict__ ent,
                                                                const unsigned char* __restrict__ mask,
                                                                int* __restrict__ ent_next, int* __restrict__ s0) {
    constexpr int NW = kBlockThreads / 64;
    __shared__ int base[8], wcnt[NW][8], early[8];
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    const int wave = threadIdx.x >> 6;
    for (int j = blockIdx.x; j < njobs; j += gridDim.x) {
        const int* J = job + 12 * j;
        const int b = J[0], len = J[1], ks = J[2];
        if (threadIdx.x < 8) { base[threadIdx.x] = 0; early[threadIdx.x] = 0; }
        __syncthreads();
        for (int chunk = 0; chunk < len; chunk += blockDim.x) {
            const int i = chunk + threadIdx.x;
            const bool in = i < len;
            const unsigned m = in ? mask[b + i] : 0u;
            const int t = in ? ent[b + i] : 0;
            int rank[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                uint64_t bal = __ballot((m >> c) & 1u);
                rank[c] = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                if (lane == 0) wcnt[wave][c] = __popcll(bal);
            }
            __syncthreads();
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (c < nchild && ((m >> c) & 1u)) {
                    int pos = base[c] + rank[c];
                    for (int w = 0; w < wave; ++w) pos += wcnt[w][c];
                    ent_next[J[3 + c] + pos] = t;
                    if (i < ks) atomicAdd(&early[c], 1);
                }
            }
            __syncthreads();
            if (threadIdx.x < 8) {
                int s = 0;
                for (int w = 0; w < NW; ++w) s += wcnt[w][threadIdx.x];
                base[threadIdx.x] += s;
            }
            __syncthreads();
        }
        if (threadIdx.x < 8) s0[8 * j + threadIdx.x] = early[threadIdx.x];
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_oct_classify(hipStream_t st, int nnodes, const float* cbox, const int* seg, const int* ent,
                               const float* tri9, unsigned char* mask, int* stats) {
    if (nnodes <= 0) return hipSuccess;
    int g = nnodes < 65536 ? nnodes : 65536;
    hipLaunchKernelGGL(k_oct_classify, dim3(g), dim3(kBlockThreads), 0, st, nnodes, cbox, seg, ent, tri9, mask, stats);
    return hipGetLastError();
}

hipError_t launch_oct_scatter(hipStream_t st, int njobs, int nchild, const int* job, const int* ent,
                              const unsigned char* mask, int* ent_next, int* s0) {
    if (njobs <= 0) return hipSuccess;
    int g = njobs < 65536 ? njobs : 65536;
    hipLaunchKernelGGL(k_oct_scatter, dim3(g), dim3(kBlockThreads), 0, st, njobs, nchild, job, ent, mask, ent_next, s0);
    return hipGetLastError();
}

}  // namespace rtmi
