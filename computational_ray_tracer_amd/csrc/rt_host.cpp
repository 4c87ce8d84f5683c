// librtmi355x — host side of the drop-in C-ABI (include/rtmi355x.h).
//
// Owns: the HIP context/stream, the scene preparation the reference does on the host before its render loop
// (TriModel world transform + back-face flags, Shapes.h:1282-1380; Octtree_Model::CreateOcttree with the
// Möller overlap test, Octtree_Model.h:33-63/180-367, AABB_triangle_Moller.h:187-474; Spectra::Init,
// spectrum.cpp:2612-2634), the flattening of that octree into the HBM layout of rt_internal.h, and the
// orchestration of the wavefront kernels of rt_kernels.hip for one render pass.
//
// There is no CPU fallback: every pass runs on the MI355X; rt_create fails without a gfx950 device.
#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <queue>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/rtmi355x.h"
#include "../data/spectra_data.h"
#include "../data/sensor_data.h"
#include "rt_guard.h"
#include "rt_internal.h"

using namespace rtmi;

namespace {

constexpr int kRingMax = 1 << 16;  // largest BFS group FIFO (HBM ring per resident thread, 4 B per entry)
constexpr int kMaxLights = 64;
constexpr int kDefaultLanes = 2;   // path-mode batches in flight on separate streams (RTMI_LANES overrides; 1 lane:
                                   // Cornell 1217, 2 lanes 1500, 3-4 lanes with 4 Mi-sample batches ~1150 Msamples/s)
constexpr float kClusterPadRel = 1e-5f;  // cluster-box inflation per unit of scene extent (see scene upload)

// ------------------------------------------------------------------------------ host float math
// glm operation order, float, -ffp-contract=off (same contract as the device code)
struct F3 { float x, y, z; float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); } };
inline F3 f3add(F3 a, F3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline F3 f3sub(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline F3 f3mul(F3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline float f3dot(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline F3 f3cross(F3 a, F3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
inline F3 f3norm(F3 v) { float s = 1.0f / std::sqrt(f3dot(v, v)); return f3mul(v, s); }
inline void m4v(const float* M, float x, float y, float z, float w, float o[4]) {
    for (int r = 0; r < 4; ++r) {
        float a0 = M[0 * 4 + r] * x, a1 = M[1 * 4 + r] * y, a2 = M[2 * 4 + r] * z, a3 = M[3 * 4 + r] * w;
        o[r] = (a0 + a1) + (a2 + a3);
    }
}
// The render-space bounding sphere of an analytic shape for the kernels' conservative cull (rt_device.h
// shape_culled): the object-space box of the shape (sphere: [-r, r]^2 x [zmin, zmax]; disk: [-ro, ro]^2 x {h};
// triangle: its vertices' box) through the inverse of render_to_object — the transform the exact test applies — in
// double, then centre = the box centre, radius = its half diagonal, padded by 1e-3 relative and 1e-3 (1 + |centre|)
// absolute.  A singular transform or a non-finite result disables the cull for the shape (bs[3] = inf).
void shape_bound(DevShape& d) {
    double a[4][8];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) { a[r][c] = d.r2o[c * 4 + r]; a[r][4 + c] = r == c ? 1.0 : 0.0; }
    bool ok = true;
    for (int c = 0; c < 4 && ok; ++c) {  // Gauss-Jordan with partial pivoting
        int pr = c;
        for (int r = c + 1; r < 4; ++r) if (std::fabs(a[r][c]) > std::fabs(a[pr][c])) pr = r;
        if (!(std::fabs(a[pr][c]) > 1e-30)) { ok = false; break; }
        for (int k = 0; k < 8; ++k) std::swap(a[c][k], a[pr][k]);
        const double iv = 1.0 / a[c][c];
        for (int k = 0; k < 8; ++k) a[c][k] *= iv;
        for (int r = 0; r < 4; ++r)
            if (r != c) { const double f = a[r][c]; for (int k = 0; k < 8; ++k) a[r][k] -= f * a[c][k]; }
    }
    double lo[3], hi[3];
    if (d.type == 0) { lo[0] = lo[1] = -d.r; hi[0] = hi[1] = d.r; lo[2] = d.zmin; hi[2] = d.zmax; }
    else if (d.type == 1) { lo[0] = lo[1] = -d.ro; hi[0] = hi[1] = d.ro; lo[2] = hi[2] = d.h; }
    else {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(std::min(d.p1[k], d.p2[k]), d.p3[k]);
            hi[k] = std::max(std::max(d.p1[k], d.p2[k]), d.p3[k]);
        }
    }
    double wlo[3] = {1e300, 1e300, 1e300}, whi[3] = {-1e300, -1e300, -1e300};
    for (int corner = 0; corner < 8 && ok; ++corner) {
        const double p[3] = {(corner & 1) ? hi[0] : lo[0], (corner & 2) ? hi[1] : lo[1], (corner & 4) ? hi[2] : lo[2]};
        for (int r = 0; r < 3; ++r) {
            const double w = a[r][4] * p[0] + a[r][5] * p[1] + a[r][6] * p[2] + a[r][7];
            wlo[r] = std::min(wlo[r], w);
            whi[r] = std::max(whi[r], w);
        }
    }
    double c[3], h2 = 0.0, cm = 0.0;
    for (int r = 0; r < 3; ++r) {
        c[r] = 0.5 * (wlo[r] + whi[r]);
        h2 += 0.25 * (whi[r] - wlo[r]) * (whi[r] - wlo[r]);
        cm = std::max(cm, std::fabs(c[r]));
    }
    const double rp = std::sqrt(h2) * 1.001 + 1e-3 * (1.0 + cm);
    for (int r = 0; r < 3; ++r) d.bs[r] = (float)c[r];
    d.bs[3] = (float)(rp * rp);
    if (!ok || !std::isfinite(d.bs[0]) || !std::isfinite(d.bs[1]) || !std::isfinite(d.bs[2]) || !std::isfinite(d.bs[3]))
        d.bs[3] = std::numeric_limits<float>::infinity();
}
inline F3 m3v(const float* M, F3 v) {
    float o[3];
    for (int r = 0; r < 3; ++r) o[r] = (M[0 * 3 + r] * v.x + M[1 * 3 + r] * v.y) + M[2 * 3 + r] * v.z;
    return {o[0], o[1], o[2]};
}

// ---------------------------------------------------------------------------------- spectra (host)
// spectrum.cpp:60-71 PiecewiseLinearSpectrum::Query with helpers.h:159-172 FindInterval
struct PLS {
    std::vector<float> l, v;
    float query(float lambda) const {
        if (l.empty() || lambda < l.front() || lambda > l.back()) return 0;
        long size = (long)l.size() - 2, first = 1;
        while (size > 0) {
            long half = size >> 1, middle = first + half;
            bool r = l[middle] <= lambda;
            first = r ? middle + 1 : first;
            size = r ? size - (half + 1) : half;
        }
        long o = std::min(std::max(first - 1, 0L), (long)l.size() - 2);
        float t = (lambda - l[o]) / (l[o + 1] - l[o]);
        return (1 - t) * v[o] + t * v[o + 1];
    }
};
struct DenseS {
    std::vector<float> v;  // 360..830
    float query(float lambda) const {
        long off = std::lround(lambda) - 360;
        return (off < 0 || off >= (long)v.size()) ? 0.f : v[off];
    }
};
template <class S>
DenseS to_dense(const S& s) {
    DenseS d;
    d.v.resize(kSpecN);
    for (int l = 360; l <= 830; ++l) d.v[l - 360] = s.query((float)l);
    return d;
}
template <class A, class B>
float inner_product(const A& f, const B& g) {  // spectrum.h:762-768
    float acc = 0;
    for (float lambda = 360; lambda <= 830; ++lambda) acc += f.query(lambda) * g.query(lambda);
    return acc;
}
struct HostSpectra {
    DenseS X, Y, Z, D65d;
    PLS D65, F1, BK7;
    PLS interleaved(const float* s, int n, bool normalize) const {  // spectrum.cpp:134-165 FromInterleaved
        PLS p;
        if (s[0] > 360) { p.l.push_back(359); p.v.push_back(s[1]); }
        for (int i = 0; i < n / 2; ++i) { p.l.push_back(s[2 * i]); p.v.push_back(s[2 * i + 1]); }
        if (p.l.back() < 830) { p.l.push_back(831); p.v.push_back(p.v.back()); }
        if (normalize) {
            float sc = 106.856895f / inner_product(p, Y);
            for (float& x : p.v) x *= sc;
        }
        return p;
    }
    void init() {
        auto cie = [](const float* t) {
            PLS p;
            p.l.assign(rtdata::cie_lambda, rtdata::cie_lambda + 471);
            p.v.assign(t, t + 471);
            return to_dense(p);
        };
        X = cie(rtdata::cie_x); Y = cie(rtdata::cie_y); Z = cie(rtdata::cie_z);
        D65 = interleaved(rtdata::illum_d65, rtdata::illum_d65_n, true);
        F1 = interleaved(rtdata::illum_f1, rtdata::illum_f1_n, true);
        BK7 = interleaved(rtdata::glass_bk7_eta, rtdata::glass_bk7_eta_n, false);  // spectrum.cpp:2674-2675
        D65d = to_dense(D65);
    }
};

// ------------------------------------------------------------------ Möller triangle / box overlap (host)
// AABB_triangle_Moller.h:187-474 (AxisTest_Z0 never rejects: the quirk at :342 is kept)
bool axis_ok(float pa, float pb, float rad) {
    float mn, mx;
    if (pa < pb) { mn = pa; mx = pb; } else { mn = pb; mx = pa; }
    return !(mn > rad || mx < -rad);
}
bool axis_ok_z12(float p1, float p2, float rad) {
    float mn, mx;
    if (p2 < p1) { mn = p2; mx = p1; } else { mn = p1; mx = p2; }
    return !(mn > rad || mx < -rad);
}
bool tri_box_overlap(F3 c, F3 h, F3 t0, F3 t1, F3 t2) {
    F3 v0 = f3sub(t0, c), v1 = f3sub(t1, c), v2 = f3sub(t2, c);
    F3 e0 = f3sub(v1, v0), e1 = f3sub(v2, v1), e2 = f3sub(v0, v2);
    float fex, fey, fez;
    fex = std::fabs(e0.x); fey = std::fabs(e0.y); fez = std::fabs(e0.z);
    if (!axis_ok(e0.z * v0.y - e0.y * v0.z, e0.z * v2.y - e0.y * v2.z, fez * h.y + fey * h.z)) return false;   // X01
    if (!axis_ok(-e0.z * v0.x + e0.x * v0.z, -e0.z * v2.x + e0.x * v2.z, fez * h.x + fex * h.z)) return false; // Y02
    if (!axis_ok_z12(e0.y * v1.x - e0.x * v1.y, e0.y * v2.x - e0.x * v2.y, fey * h.x + fex * h.y)) return false; // Z12
    fex = std::fabs(e1.x); fey = std::fabs(e1.y); fez = std::fabs(e1.z);
    if (!axis_ok(e1.z * v0.y - e1.y * v0.z, e1.z * v2.y - e1.y * v2.z, fez * h.y + fey * h.z)) return false;   // X01
    if (!axis_ok(-e1.z * v0.x + e1.x * v0.z, -e1.z * v2.x + e1.x * v2.z, fez * h.x + fex * h.z)) return false; // Y02
    // Z0: never rejects (reference returns true on both paths)
    fex = std::fabs(e2.x); fey = std::fabs(e2.y); fez = std::fabs(e2.z);
    if (!axis_ok(e2.z * v0.y - e2.y * v0.z, e2.z * v1.y - e2.y * v1.z, fez * h.y + fey * h.z)) return false;   // X2
    if (!axis_ok(-e2.z * v0.x + e2.x * v0.z, -e2.z * v1.x + e2.x * v1.z, fez * h.x + fex * h.z)) return false; // Y1
    if (!axis_ok_z12(e2.y * v1.x - e2.x * v1.y, e2.y * v2.x - e2.x * v2.y, fey * h.x + fex * h.y)) return false; // Z12
    auto mm = [](float a, float b, float c, float& mn, float& mx) {
        mn = mx = a;
        if (b < mn) mn = b;
        if (b > mx) mx = b;
        if (c < mn) mn = c;
        if (c > mx) mx = c;
    };
    float mn, mx;
    mm(v0.x, v1.x, v2.x, mn, mx);
    if (mn > h.x || mx < -h.x) return false;
    mm(v0.y, v1.y, v2.y, mn, mx);
    if (mn > h.y || mx < -h.y) return false;
    mm(v0.z, v1.z, v2.z, mn, mx);
    if (mn > h.z || mx < -h.z) return false;
    F3 nrm = f3cross(e0, e1);  // planeBoxOverlap
    float vmin[3], vmax[3];
    for (int q = 0; q < 3; ++q) {
        float v = v0[q], nq = nrm[q], mb = h[q];
        if (nq > 0.0f) { vmin[q] = -mb - v; vmax[q] = mb - v; }
        else { vmin[q] = mb - v; vmax[q] = -mb - v; }
    }
    if (f3dot(nrm, {vmin[0], vmin[1], vmin[2]}) > 0.0f) return false;
    if (f3dot(nrm, {vmax[0], vmax[1], vmax[2]}) >= 0.0f) return true;
    return false;
}

// ------------------------------------------------------------------------------- octree builder
// Octtree_Model.h:33-63 CreateOcttree, 180-277 AddTriangle, 279-358 Split, 361-367 tri_boundsIntersection
struct OctBuild {
    struct Node { F3 mn, mx; int first_child = -1; std::vector<int> tris; };
    std::vector<Node> nodes;
    const std::vector<F3>* tri3 = nullptr;  // 3 world vertices per triangle
    int capacity = 40;

    bool overlap(int t, const Node& n) const {
        F3 half = {(n.mx.x - n.mn.x) / 2.0f, (n.mx.y - n.mn.y) / 2.0f, (n.mx.z - n.mn.z) / 2.0f};
        F3 c = f3add(n.mn, half);
        const F3* p = &(*tri3)[3 * (size_t)t];
        return tri_box_overlap(c, half, p[0], p[1], p[2]);
    }
    // the 8 padded child boxes of a node (Octtree_Model.h:279-300): top fl, fr, bl, br, bottom fl, fr, bl, br
    static void child_boxes(F3 mn, F3 mx, F3 cmn[8], F3 cmx[8]) {
        F3 h = {(mx.x - mn.x) / 2.0f, (mx.y - mn.y) / 2.0f, (mx.z - mn.z) / 2.0f};
        F3 C = f3add(mn, h);
        h = f3add(h, {0.01f, 0.01f, 0.01f});
        const F3 lo[8] = {{-h.x, 0, -h.z}, {0, 0, -h.z}, {-h.x, 0, 0}, {0, 0, 0},
                          {-h.x, -h.y, -h.z}, {0, -h.y, -h.z}, {-h.x, -h.y, 0}, {0, -h.y, 0}};
        const F3 hi[8] = {{0, h.y, 0}, {h.x, h.y, 0}, {0, h.y, h.z}, {h.x, h.y, h.z},
                          {0, 0, 0}, {h.x, 0, 0}, {0, 0, h.z}, {h.x, 0, h.z}};
        for (int k = 0; k < 8; ++k) { cmn[k] = f3add(C, lo[k]); cmx[k] = f3add(C, hi[k]); }
    }
    void split(int id) {
        Node ch[8];
        {
            F3 cmn[8], cmx[8];
            child_boxes(nodes[id].mn, nodes[id].mx, cmn, cmx);
            for (int k = 0; k < 8; ++k) { ch[k].mn = cmn[k]; ch[k].mx = cmx[k]; }
        }
        for (int t : nodes[id].tris)
            for (int k = 0; k < 8; ++k)
                if (overlap(t, ch[k])) ch[k].tris.push_back(t);
        size_t cnt = nodes[id].tris.size();
        for (int k = 0; k < 8; ++k)
            if (ch[k].tris.size() == cnt) return;  // abort rule (Octtree_Model.h:331-340)
        int first = (int)nodes.size();
        for (int k = 0; k < 8; ++k) nodes.push_back(std::move(ch[k]));
        nodes[id].first_child = first;
        nodes[id].tris.clear();
        nodes[id].tris.shrink_to_fit();
    }
    void add(int t) {
        std::queue<int> q;
        q.push(0);
        while (!q.empty()) {
            int cur = q.front();
            q.pop();
            if (!overlap(t, nodes[cur])) continue;
            if (nodes[cur].first_child < 0) {
                nodes[cur].tris.push_back(t);
                if ((int)nodes[cur].tris.size() >= capacity) split(cur);
            } else {
                for (int k = 0; k < 8; ++k) q.push(nodes[cur].first_child + k);
            }
        }
    }
};

// On-device build of the same tree (rt_octree.hip: the level-synchronous form of the sequential insertion).  The
// device classifies and scatters each level; the host decides the splits (k = max(capacity, s0 + 1, M + 1) <= len),
// lays out the next level in BFS order and at the end renumbers the nodes in the order the sequential build
// creates them: by the triangle whose insertion triggered the split, then BFS order within that insertion.
int octree_build_device(hipStream_t st, OctBuild& ob, int nt, std::string& err) {
    struct LNode {
        F3 mn, mx;
        int begin, len, s0, level;
        int first_child = -1, trigger = -1;
    };
    auto ok = [&](hipError_t e, const char* what) {
        if (e != hipSuccess) err = std::string("octree build: ") + what + ": " + hipGetErrorString(e);
        return e == hipSuccess;
    };
    std::vector<void*> owned;
    auto dmalloc = [&](void** p, size_t bytes) {
        hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
        if (e == hipSuccess) owned.push_back(*p);
        return e;
    };
    struct Free {
        std::vector<void*>& v;
        ~Free() { for (void* p : v) hipFree(p); }
    } free_all{owned};
    const std::vector<F3>& tri3 = *ob.tri3;
    float* d_tri9 = nullptr;
    int *d_ent = nullptr, *d_seg = nullptr, *d_stats = nullptr, *d_job = nullptr, *d_s0 = nullptr;
    unsigned char* d_mask = nullptr;
    float* d_cbox = nullptr;
    if (!ok(dmalloc((void**)&d_tri9, sizeof(F3) * tri3.size()), "alloc") ||
        !ok(hipMemcpyAsync(d_tri9, tri3.data(), sizeof(F3) * tri3.size(), hipMemcpyHostToDevice, st), "upload"))
        return RT_E_HIP;
    // root pass: A_root = the triangles overlapping the root box, in insertion order
    std::vector<int> iota(nt);
    for (int t = 0; t < nt; ++t) iota[t] = t;
    size_t cap_ent = std::max<size_t>(nt, 1), cap_nodes = 1, cap_mask = cap_ent;
    int* d_next = nullptr;
    if (!ok(dmalloc((void**)&d_ent, 4 * cap_ent), "alloc") || !ok(dmalloc((void**)&d_next, 4 * cap_ent), "alloc") ||
        !ok(dmalloc((void**)&d_mask, cap_ent), "alloc") || !ok(dmalloc((void**)&d_cbox, 4 * 48), "alloc") ||
        !ok(dmalloc((void**)&d_seg, 4 * 2), "alloc") || !ok(dmalloc((void**)&d_stats, 4 * 9), "alloc") ||
        !ok(dmalloc((void**)&d_job, 4 * 12), "alloc") || !ok(dmalloc((void**)&d_s0, 4 * 8), "alloc"))
        return RT_E_OOM;
    {
        float box[48];
        const F3 rmn = ob.nodes[0].mn, rmx = ob.nodes[0].mx;
        for (int k = 0; k < 8; ++k) {
            box[6 * k] = rmn.x; box[6 * k + 1] = rmn.y; box[6 * k + 2] = rmn.z;
            box[6 * k + 3] = rmx.x; box[6 * k + 4] = rmx.y; box[6 * k + 5] = rmx.z;
        }
        int seg[2] = {0, nt}, job[12] = {0, nt, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stats[9];
        if (!ok(hipMemcpyAsync(d_ent, iota.data(), 4 * (size_t)nt, hipMemcpyHostToDevice, st), "upload") ||
            !ok(hipMemcpyAsync(d_cbox, box, sizeof(box), hipMemcpyHostToDevice, st), "upload") ||
            !ok(hipMemcpyAsync(d_seg, seg, sizeof(seg), hipMemcpyHostToDevice, st), "upload") ||
            !ok(hipMemcpyAsync(d_job, job, sizeof(job), hipMemcpyHostToDevice, st), "upload") ||
            !ok(launch_oct_classify(st, 1, d_cbox, d_seg, d_ent, d_tri9, d_mask, d_stats), "classify") ||
            !ok(launch_oct_scatter(st, 1, 1, d_job, d_ent, d_mask, d_next, d_s0), "scatter") ||
            !ok(hipMemcpyAsync(stats, d_stats, sizeof(stats), hipMemcpyDeviceToHost, st), "download") ||
            !ok(hipStreamSynchronize(st), "sync"))
            return RT_E_HIP;
        std::swap(d_ent, d_next);
        LNode root{rmn, rmx, 0, stats[1], 0, 0};
        ob.nodes.clear();
        std::vector<LNode> all{root};
        std::vector<std::vector<int>> level_ents;
        std::vector<int> frontier{0};
        size_t cap_next = cap_ent;
        while (!frontier.empty()) {
            const int n = (int)frontier.size();
            std::vector<float> cbox(48 * (size_t)n);
            std::vector<int> segs(2 * (size_t)n);
            int total = 0;
            for (int i = 0; i < n; ++i) {
                const LNode& N = all[frontier[i]];
                F3 cmn[8], cmx[8];
                OctBuild::child_boxes(N.mn, N.mx, cmn, cmx);
                for (int k = 0; k < 8; ++k) {
                    float* q = &cbox[48 * (size_t)i + 6 * k];
                    q[0] = cmn[k].x; q[1] = cmn[k].y; q[2] = cmn[k].z; q[3] = cmx[k].x; q[4] = cmx[k].y; q[5] = cmx[k].z;
                }
                segs[2 * i] = N.begin; segs[2 * i + 1] = N.len;
                total = std::max(total, N.begin + N.len);
            }
            if ((size_t)n > cap_nodes) {
                cap_nodes = 2 * (size_t)n;
                for (void* p : {(void*)d_cbox, (void*)d_seg, (void*)d_stats, (void*)d_job, (void*)d_s0}) {
                    hipFree(p);
                    owned.erase(std::find(owned.begin(), owned.end(), p));
                }
                if (!ok(dmalloc((void**)&d_cbox, 4 * 48 * cap_nodes), "alloc") ||
                    !ok(dmalloc((void**)&d_seg, 4 * 2 * cap_nodes), "alloc") ||
                    !ok(dmalloc((void**)&d_stats, 4 * 9 * cap_nodes), "alloc") ||
                    !ok(dmalloc((void**)&d_job, 4 * 12 * cap_nodes), "alloc") ||
                    !ok(dmalloc((void**)&d_s0, 4 * 8 * cap_nodes), "alloc"))
                    return RT_E_OOM;
            }
            if ((size_t)total > cap_mask) {  // one mask byte per entry of the largest level
                cap_mask = 2 * (size_t)total;
                hipFree(d_mask);
                owned.erase(std::find(owned.begin(), owned.end(), (void*)d_mask));
                if (!ok(dmalloc((void**)&d_mask, cap_mask), "alloc")) return RT_E_OOM;
            }
            std::vector<int> stats(9 * (size_t)n);
            level_ents.emplace_back((size_t)total);
            if (!ok(hipMemcpyAsync(d_cbox, cbox.data(), 4 * cbox.size(), hipMemcpyHostToDevice, st), "upload") ||
                !ok(hipMemcpyAsync(d_seg, segs.data(), 4 * segs.size(), hipMemcpyHostToDevice, st), "upload") ||
                !ok(launch_oct_classify(st, n, d_cbox, d_seg, d_ent, d_tri9, d_mask, d_stats), "classify") ||
                !ok(hipMemcpyAsync(stats.data(), d_stats, 4 * stats.size(), hipMemcpyDeviceToHost, st), "download") ||
                !ok(hipMemcpyAsync(level_ents.back().data(), d_ent, 4 * (size_t)total, hipMemcpyDeviceToHost, st),
                    "download") ||
                !ok(hipStreamSynchronize(st), "sync"))
                return RT_E_HIP;
            // splits, in frontier (BFS) order; children laid out contiguously in the next level's sequence array
            std::vector<int> jobs, next_frontier;
            int running = 0;
            for (int i = 0; i < n; ++i) {
                LNode& N = all[frontier[i]];
                const int* S = &stats[9 * (size_t)i];
                int k = std::max(std::max(ob.capacity, N.s0 + 1), S[0] + 1);
                if (k > N.len) continue;
                N.trigger = level_ents.back()[(size_t)N.begin + k - 1];
                N.first_child = (int)all.size();
                int job[12] = {N.begin, N.len, k, 0, 0, 0, 0, 0, 0, 0, 0, 0};
                F3 cmn[8], cmx[8];
                OctBuild::child_boxes(N.mn, N.mx, cmn, cmx);
                const int lvl = N.level;
                for (int c = 0; c < 8; ++c) {
                    job[3 + c] = running;
                    all.push_back(LNode{cmn[c], cmx[c], running, S[1 + c], 0, lvl + 1});
                    next_frontier.push_back((int)all.size() - 1);
                    running += S[1 + c];
                }
                jobs.insert(jobs.end(), job, job + 12);
            }
            if (jobs.empty()) break;
            const int nj = (int)jobs.size() / 12;
            if ((size_t)running > cap_next) {
                cap_next = 2 * (size_t)running;
                hipFree(d_next);
                owned.erase(std::find(owned.begin(), owned.end(), (void*)d_next));
                if (!ok(dmalloc((void**)&d_next, 4 * cap_next), "alloc")) return RT_E_OOM;
            }
            std::vector<int> s0(8 * (size_t)nj);
            if (!ok(hipMemcpyAsync(d_job, jobs.data(), 4 * jobs.size(), hipMemcpyHostToDevice, st), "upload") ||
                !ok(launch_oct_scatter(st, nj, 8, d_job, d_ent, d_mask, d_next, d_s0), "scatter") ||
                !ok(hipMemcpyAsync(s0.data(), d_s0, 4 * s0.size(), hipMemcpyDeviceToHost, st), "download") ||
                !ok(hipStreamSynchronize(st), "sync"))
                return RT_E_HIP;
            for (int j = 0; j < nj; ++j)
                for (int c = 0; c < 8; ++c) all[next_frontier[8 * j + c]].s0 = s0[8 * (size_t)j + c];
            std::swap(d_ent, d_next);
            std::swap(cap_ent, cap_next);
            frontier.swap(next_frontier);
        }
        // renumber: the sequential build appends a split node's 8 children when its trigger triangle is inserted
        std::vector<int> splits;
        for (int i = 0; i < (int)all.size(); ++i)
            if (all[i].first_child >= 0) splits.push_back(i);
        std::stable_sort(splits.begin(), splits.end(), [&](int a, int b) { return all[a].trigger < all[b].trigger; });
        std::vector<int> seq(all.size(), -1);
        seq[0] = 0;
        for (size_t r = 0; r < splits.size(); ++r)
            for (int c = 0; c < 8; ++c) seq[all[splits[r]].first_child + c] = 1 + 8 * (int)r + c;
        ob.nodes.assign(all.size(), OctBuild::Node{});
        for (int i = 0; i < (int)all.size(); ++i) {
            const LNode& N = all[i];
            OctBuild::Node& o = ob.nodes[seq[i]];
            o.mn = N.mn; o.mx = N.mx;
            if (N.first_child >= 0) {
                o.first_child = seq[N.first_child];
            } else {
                const std::vector<int>& E = level_ents[N.level];
                o.tris.assign(E.begin() + N.begin, E.begin() + N.begin + N.len);
            }
        }
    }
    return RT_OK;
}

// ---------------------------------------------------------------------------------------- buffers
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
};

}  // namespace

// The device buffers of one batch in flight (grown on demand).  Path mode keeps kLanes of them so that consecutive
// batches run concurrently on separate streams: one batch's VALU-bound traversal overlaps the other's HBM-bound
// path-state traffic.
static const int kLanes = 4;
struct Work {
    size_t cap = 0;
    float4 *rayO = nullptr, *rayD = nullptr, *lamA = nullptr, *lamB = nullptr, *pdfA = nullptr, *pdfB = nullptr;
    float4* hitB = nullptr;
    float4* rec = nullptr;     // path mode: one 128-B record per slot (rt_internal.h R_*)
    int* hitPrim = nullptr;
    int* d_qcount = nullptr;   // queue q's counters at [q * kQRegion + kQLen / kQTraceTicket / ...] (rt_internal.h)
    // coherence sort of path queues (multi-level octrees): side queue, radix-sort buffers
    float4 *sO = nullptr, *sD = nullptr;
    int *sS = nullptr, *sVals = nullptr, *sValsAlt = nullptr;  // sS: the sort permutation (TraceIO perm)
    unsigned *sKeys = nullptr, *sKeysAlt = nullptr;
    unsigned* sQKey = nullptr;  // the ray queue's sort keys at queue positions (written by the shade kernels)
    void* sTemp = nullptr;      // the sorts' histograms and meta (sort_temp_bytes)
    size_t sCap = 0;
    // shadow queue (multi-level octrees): {o, tMax}, {d, slot}, pending contribution (2 x float4)
    float4 *shO = nullptr, *shD = nullptr, *shLA = nullptr, *shLB = nullptr;
    size_t shCap = 0;
    // deferred NEE of the mixed-scene shade (rt_internal.h NeeIO): records per slot, the NEE queue's slots
    float4* neeRec = nullptr;
    int* neeSlot = nullptr;
    size_t neeRecCap = 0, neeSlotCap = 0;  // float4s, ints
    // BFS FIFO overflow ring of the multi-level traversal (qcap 0): one per lane, because the lanes' kernels run
    // concurrently and index the ring by their own global thread id
    int* ring = nullptr;
    size_t ring_cap = 0;   // ints
    // multi-level scenes in path mode: the queue positions of the rays the trace kernel's BVH walk could not decide
    // (TraceIO fb_pos; k_trace_fallback traces them with the reference BFS)
    int* tfb = nullptr;
    size_t tfb_cap = 0;    // ints
    hipStream_t stream = nullptr;  // lanes >= 1: own stream (lane 0 runs on the caller's stream)
    hipEvent_t film_done = nullptr;
};

struct rt_ctx {
    // coherence sort of path queues (multi-level octrees): scene quantisation of the sort key
    float4 sort_lo{}, sort_scale{};
    int device = 0;
    int octree_build = RT_OCTREE_BUILD_DEVICE;
    hipStream_t stream = nullptr;
    std::string err;
    bool have_scene = false, have_cam = false, have_smp = false, have_film = false, have_integ = false;
    rt_camera_desc cam{};
    rt_sampler_desc smp{};
    rt_film_desc film{};
    rt_integrator_desc integ{};
    // scene (host mirrors kept for export)
    int n_tris = 0;
    std::vector<float> h_bounds;
    std::vector<int32_t> h_child, h_leaf_first, h_leaf_count, h_refs;
    rt_octree_info info{};
    bool cull = false;
    bool scene_full = false;   // the scene needs the general path-shade kernel
    DevScene dsc{};
    std::vector<void*> scene_allocs;
    // spectra + resolve matrices
    HostSpectra hs;
    DevSpectra* d_spec = nullptr;
    float resolveA[9], resolveB[9];
    float* d_resolve = nullptr;
    // pixel work list
    int tile = 32, n_shards = 1, shard_id = 0;
    bool work_dirty = true;
    int n_work = 0;
    int* d_work = nullptr;
    // batch workspaces, one per lane (path mode runs kLanes batches concurrently on separate streams)
    Work ws[kLanes];
    bool warned_eye = false;    // check_ready: the camera-eye-beyond-oguard warning was printed
    bool stage_events = true;   // per-stage HIP events (rt_stats ms_*); RTMI_NO_STAGE_EVENTS=1 turns them off
    int lanes = kDefaultLanes;  // batches in flight in path mode (RTMI_LANES overrides)
    // multi-level simple path scenes: NEE rays traced by k_path_shadow (RTMI_SHADOW_QUEUE=1; measured slower than
    // the inline any-hit, kept as a parity-tested option), depth first (RTMI_SHADOW_DFS, exact any-hit, §6)
    int shadow_queue = 0;
    int shadow_dfs = 1;
    int sort_rays = 1;         // RTMI_SORT=0: no coherence sort (A/B)
    float bvh_node_cost = 2.5f;  // SAH node cost relative to a triangle test (RTMI_BVH_CI; r04 with 64 bins: 2.5 vs 3 CFG3 +1.6 %, CFG4 +1.2 %)
    int bvh_max_leaf = kBvhMaxLeaf;  // triangles per BVH leaf at most (RTMI_BVH_LEAF)
    int bvh_count[3][2] = {};  // per BVH (set 0, set 1, any-hit): nodes, tiles (rt_bvh_export)
    // the any-hit walks' BVH: its own (SAH node cost 2, leaves <= 4), or with RTMI_BVH_ANY="0/4" the closest-hit BVH
    // of set 0 itself (one working set for both queries).  r04 A/B: the shared BVH made CFG4's NEE stage 7.7 % slower
    // (30.0 vs 27.9 ms per step): the shadow rays' better tree outweighs the smaller working set
    float bvh_any_cost = 2.f;
    int bvh_any_leaf = 4;
    int force_amb = -1;        // RTMI_FORCE_AMB=k (test knob, DevScene amb_force / amb_mask): -1 off
    int coop = 1;              // RTMI_COOP=0 (test knob): undecided rays to the fallback kernels (DevScene coop_ok 0)
    int mat_bins = 1;          // RTMI_MAT_BINS=0: mixed multi-level scenes shade every material in one kernel (A/B)
    int emit_filter = 1;       // RTMI_EMIT_FILTER=0: the last depth of a mixed scene traces every ray (A/B)
    int debug_path = 0;        // RTMI_DEBUG_PATH_KERNELS=1 (tests): rt_debug_trace / _occluded run path mode's kernels
    int sort_dir_bits = 3, sort_org_bits = 3;  // sort key widths (RTMI_SORT_BITS="dir/org[/major]"; r03 A/B: 3/3 vs 3/4 CFG3 +1 %, 2/3 -4 %)
    // origin Morton code in the key's high bits (1) or the direction (0); -1: origin-major on the simple path, whose
    // shade kernel traces the NEE shadow rays inline (CFG3 588 -> 600), direction-major in mixed scenes, whose NEE
    // queue has a sort of its own (CFG4 372 vs 367)
    int sort_org_major = -1;
    // Morton sort of the NEE queue (mixed multi-level scenes; RTMI_SORT_NEE="on[/bits]"): CFG4 337 -> 364 at 9 bits
    // per axis (6 / 7 bits: 353 / 356; CFG5 334 -> 355 at 7)
    int sort_nee = 1, sort_nee_bits = 8;  // (r03, device radix sort: 8 bits = 3 passes, CFG4 +1.5 % over 9 bits = 4 passes)
    hipEvent_t done = nullptr; // recorded at the end of every pass: a later call on another stream waits for it
    size_t batch_samples = 0;  // samples in flight per batch (0: 16 Mi single leaf, 32 Mi multi-level; RTMI_BATCH_SAMPLES)
    unsigned long long* d_ctr = nullptr;
    float4* d_film = nullptr;  // staging film for rt_render_pass (host film)
    float* d_cdf = nullptr;    // Gaussian / Lanczos filter tables: x then y, cdf_n + 1 floats each
    int cdf_n = 0;
    int film_y_int = 0;  // the film's raster y (float division + floor) equals the integer division for every pixel
    uint32_t* d_sobol_mats = nullptr;  // Sobol generator columns; d_sobol_fwd: fwd then inv tables for sobol_m
    uint64_t* d_sobol_fwd = nullptr;
    int sobol_m = 0;
    size_t film_cap = 0;
    int grid = 0;              // persistent grid size (blocks)
    // stats
    rt_stats stats{};
    struct Ev { hipEvent_t a, b; int stage; };
    std::vector<Ev> pending;
    std::vector<hipEvent_t> pool;
    int work_epoch = 0;        // bumped whenever build_work rebuilds d_work
    // multi-device context (rt_options.n_devices > 1): this context renders on devices[0] and
    // peers[j] on devices[j + 1]; tile t of the caller's shard goes to device (t / n_shards) mod n_devices
    std::vector<rt_ctx*> peers;
    struct PeerLink {          // on devices[0]: peer j's owned pixel ids and its compact exchange buffer
        int* work0 = nullptr;
        float4* xfer0 = nullptr;
        size_t cap = 0;
        int n = 0, epoch = -1;
    };
    std::vector<PeerLink> links;
    hipEvent_t gathered = nullptr;   // devices[0]: peers' pixels packed (multi-device) / peer: pass done
    float4* xfer = nullptr;          // on a peer: its compact exchange buffer
    size_t xfer_cap = 0;
};

namespace {

// RTMI_BVH_ANY = "cost/leaf" (both fields required; anything else keeps the defaults): the any-hit BVH's SAH node cost
// and largest leaf, cost 0 = the closest-hit BVH of set 0 itself.  One parser for rt_create and rt_debug_bvh_build, so
// the exported and the uploaded any-hit BVHs come from the same parameters.
void parse_bvh_any(float& cost, int& leaf) {
    const char* e = std::getenv("RTMI_BVH_ANY");
    float ac;
    int al;
    if (e && std::sscanf(e, "%f/%d", &ac, &al) == 2) {
        cost = ac;
        leaf = std::max(1, std::min(15, al));
    }
}

void set_error(rt_ctx* c, const std::string& msg) {
    if (c) c->err = msg;
}
int fail(rt_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}
#define HIPCHK(c, call)                                                                                   \
    do {                                                                                                  \
        hipError_t _e = (call);                                                                           \
        if (_e != hipSuccess)                                                                             \
            return fail((c), _e == hipErrorOutOfMemory ? RT_E_OOM : RT_E_HIP,                             \
                        std::string(#call) + ": " + hipGetErrorString(_e));                               \
    } while (0)

template <class T>
hipError_t dalloc(T** p, size_t n) {
    return hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T));
}

void free_scene(rt_ctx* c) {
    for (void* p : c->scene_allocs) hipFree(p);
    c->scene_allocs.clear();
    c->dsc = DevScene{};
    c->have_scene = false;
}

void free_shadow_workspace(Work& w) {
    void* ptrs[] = {w.shO, w.shD, w.shLA, w.shLB, w.neeRec, w.neeSlot};
    for (void* p : ptrs)
        if (p) hipFree(p);
    w.shO = w.shD = w.shLA = w.shLB = nullptr;
    w.neeRec = nullptr;
    w.neeSlot = nullptr;
    w.shCap = w.neeRecCap = w.neeSlotCap = 0;
}

int ensure_nee_workspace(rt_ctx* c, Work& w, size_t rec_f4, size_t nq) {
    if (w.neeRecCap < rec_f4) {
        if (w.neeRec) hipFree(w.neeRec);
        w.neeRec = nullptr;
        w.neeRecCap = 0;
        HIPCHK(c, dalloc(&w.neeRec, rec_f4));
        w.neeRecCap = rec_f4;
    }
    if (w.neeSlotCap < nq) {
        if (w.neeSlot) hipFree(w.neeSlot);
        w.neeSlot = nullptr;
        w.neeSlotCap = 0;
        HIPCHK(c, dalloc(&w.neeSlot, nq));
        w.neeSlotCap = nq;
    }
    return RT_OK;
}

int ensure_shadow_workspace(rt_ctx* c, Work& w, size_t n) {
    if (w.shCap >= n) return RT_OK;
    free_shadow_workspace(w);
    HIPCHK(c, dalloc(&w.shO, n)); HIPCHK(c, dalloc(&w.shD, n));
    HIPCHK(c, dalloc(&w.shLA, n)); HIPCHK(c, dalloc(&w.shLB, n));
    w.shCap = n;
    return RT_OK;
}

void free_sort_workspace(Work& w) {
    void* ptrs[] = {w.sO, w.sS, w.sVals, w.sValsAlt, w.sKeys, w.sKeysAlt, w.sQKey, w.sTemp};  // (sD = sO + 1)
    for (void* p : ptrs)
        if (p) hipFree(p);
    w.sO = w.sD = nullptr;
    w.sS = w.sVals = w.sValsAlt = nullptr;
    w.sKeys = w.sKeysAlt = w.sQKey = nullptr;
    w.sTemp = nullptr;
    w.sCap = 0;
}

int ensure_sort_workspace(rt_ctx* c, Work& w, size_t n) {
    if (w.sCap >= n) return RT_OK;
    free_sort_workspace(w);
    // the side queue's rays as interleaved (o, d) pairs like the queues' (sD = sO + 1)
    HIPCHK(c, dalloc(&w.sO, 2 * n)); w.sD = w.sO + 1; HIPCHK(c, dalloc(&w.sS, n));
    HIPCHK(c, dalloc(&w.sVals, n)); HIPCHK(c, dalloc(&w.sValsAlt, n));
    HIPCHK(c, dalloc(&w.sKeys, n)); HIPCHK(c, dalloc(&w.sKeysAlt, n)); HIPCHK(c, dalloc(&w.sQKey, n));
    HIPCHK(c, hipMalloc(&w.sTemp, sort_temp_bytes()));
    w.sCap = n;
    return RT_OK;
}

// batch buffers only (the queue counters, stream and event of a lane live as long as the context)
void free_workspace(Work& w) {
    free_sort_workspace(w);
    free_shadow_workspace(w);
    void* ptrs[] = {w.rayO, w.lamA, w.lamB, w.pdfA, w.pdfB, w.hitB, w.rec, w.hitPrim};  // (rayD = rayO + 1)
    for (void* p : ptrs)
        if (p) hipFree(p);
    w.rayO = w.rayD = w.lamA = w.lamB = w.pdfA = w.pdfB = w.hitB = w.rec = nullptr;
    w.hitPrim = nullptr;
    w.cap = 0;
}
void free_ring(Work& w) {
    if (w.ring) hipFree(w.ring);
    w.ring = nullptr;
    w.ring_cap = 0;
    if (w.tfb) hipFree(w.tfb);
    w.tfb = nullptr;
    w.tfb_cap = 0;
}
void free_workspace(rt_ctx* c) {
    for (Work& w : c->ws) {
        free_workspace(w);
        free_ring(w);
    }
}

// this lane's BFS overflow ring (multi-level octrees whose FIFO bound exceeds the register variants)
int ensure_ring(rt_ctx* c, Work& w) {
    if (c->dsc.qcap != 0) return RT_OK;
    const size_t need = (size_t)c->dsc.ring_threads * (size_t)(c->dsc.ring_mask + 1);
    if (w.ring_cap < need) {
        free_ring(w);
        HIPCHK(c, dalloc(&w.ring, need));
        w.ring_cap = need;
    }
    return RT_OK;
}
// this lane's trace-fallback list (multi-level octrees, path mode): one entry per queue position at most
int ensure_trace_fallback(rt_ctx* c, Work& w, size_t n) {
    if (w.tfb_cap >= n) return RT_OK;
    if (w.tfb) hipFree(w.tfb);
    w.tfb = nullptr;
    w.tfb_cap = 0;
    HIPCHK(c, dalloc(&w.tfb, n));
    w.tfb_cap = n;
    return RT_OK;
}
// the scene as a lane's kernels see it: its own overflow ring
DevScene lane_scene(const rt_ctx* c, const Work& w) {
    DevScene d = c->dsc;
    d.ring = w.ring;
    return d;
}

int ensure_workspace(rt_ctx* c, Work& w, size_t n, bool path) {
    int rc;
    if (!w.d_qcount) HIPCHK(c, dalloc(&w.d_qcount, 2 * kQRegion));
    if (&w != &c->ws[0]) {
        if (!w.stream) HIPCHK(c, hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
        if (!w.film_done) HIPCHK(c, hipEventCreateWithFlags(&w.film_done, hipEventDisableTiming));
    } else if (!w.film_done) {
        HIPCHK(c, hipEventCreateWithFlags(&w.film_done, hipEventDisableTiming));
    }
    if ((rc = ensure_ring(c, w))) return rc;
    if (w.cap >= n && (path ? w.rec != nullptr : w.lamA != nullptr)) return RT_OK;
    free_workspace(w);
    // path mode: queue arrays hold 2 ping-pong queues of n entries each
    size_t nq = path ? 2 * n : n;
    // rays as interleaved (o, d) pairs, 32 B per ray (rayD = rayO + 1, kernels index [k << rsh] with rsh = 1): a
    // scattered read of one ray (the coherence sort's gather) touches one line instead of two
    HIPCHK(c, dalloc(&w.rayO, 2 * nq)); w.rayD = w.rayO + 1;
    HIPCHK(c, dalloc(&w.pdfA, n)); HIPCHK(c, dalloc(&w.pdfB, n));
    HIPCHK(c, dalloc(&w.hitB, n)); HIPCHK(c, dalloc(&w.hitPrim, n));
    if (path) {
        HIPCHK(c, dalloc(&w.rec, (size_t)kRecF4 * n));
    } else {
        HIPCHK(c, dalloc(&w.lamA, n)); HIPCHK(c, dalloc(&w.lamB, n));
    }
    w.cap = n;
    return RT_OK;
}
int ensure_workspace(rt_ctx* c, size_t n, bool path) { return ensure_workspace(c, c->ws[0], n, path); }

// Sampler dimension bookkeeping of the simple path integrator (rt_device.h Smp): every path of a depth has drawn
// the same dimensions — the camera sample, then two Get2D per bounce — so the shade kernel takes its starting
// dimension as an argument instead of a per-slot field.  (A stratified sample with index >= spp draws zeros without
// advancing; its dimension is never read again.)
static int dim_get2d(const DevSampler& S, int dim) {
    if (S.kind == 1) return dim + 2;
    if (S.kind == 2) return (dim + 1 >= kSobolDims ? 2 : dim) + 2;
    return dim;
}
static int dim_after_camera(const DevSampler& S, const DevCamera& cam) {
    int dim = S.kind == 2 ? 2 : 0;                                                // StartPixelSample
    if (S.kind == 1) dim += 1;                                                    // Get1D (wavelengths)
    else if (S.kind == 2) dim = (dim >= kSobolDims ? 2 : dim) + 1;
    if (S.kind == 1) dim += 2;                                                    // GetPixel2D
    if ((cam.type == RT_CAMERA_PERSPECTIVE && cam.lens_radius > 0) || cam.type > RT_CAMERA_PINHOLE)
        dim = dim_get2d(S, dim);                                                  // lens sample
    return dim;
}

hipEvent_t ev_get(rt_ctx* c) {
    if (!c->pool.empty()) {
        hipEvent_t e = c->pool.back();
        c->pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}
void ev_mark(rt_ctx* c, hipStream_t st, int stage, hipEvent_t a) {
    if (!a) return;  // stage timing off
    hipEvent_t b = ev_get(c);
    hipEventRecord(b, st);
    c->pending.push_back({a, b, stage});
}
hipEvent_t ev_start(rt_ctx* c, hipStream_t st) {
    if (!c->stage_events) return nullptr;
    hipEvent_t a = ev_get(c);
    hipEventRecord(a, st);
    return a;
}
enum { ST_GEN = 0, ST_TRACE, ST_SHADE, ST_SHADOW, ST_FILM, ST_SORT, ST_FILTER };

void harvest(rt_ctx* c) {
    for (auto& e : c->pending) {
        float ms = 0;
        hipEventSynchronize(e.b);
        hipEventElapsedTime(&ms, e.a, e.b);
        switch (e.stage) {
            case ST_GEN: c->stats.ms_generate += ms; break;
            case ST_TRACE: c->stats.ms_trace += ms; c->stats.launches_trace += 1; break;
            case ST_SHADE: c->stats.ms_shade += ms; c->stats.launches_shade += 1; break;
            case ST_SHADOW: c->stats.ms_shadow += ms; break;
            case ST_SORT: c->stats.ms_sort += ms; break;
            case ST_FILTER: c->stats.ms_trace += ms; break;  // (the last depth's emitter filter: no trace launch)
            default: c->stats.ms_film += ms; break;
        }
        c->pool.push_back(e.a);
        c->pool.push_back(e.b);
    }
    c->pending.clear();
}

// Owned pixels in tile order: tile_size² tiles in row-major tile order, tile t owned iff t % n == id;
// inside a tile 8×8 micro-tiles (one wave64 = one micro-tile → coherent rays), row-major inside.
int build_work(rt_ctx* c) {
    if (!c->work_dirty && c->d_work) return RT_OK;
    int W = c->film.res_x, H = c->film.res_y, T = c->tile;
    int tx = (W + T - 1) / T, ty = (H + T - 1) / T;
    std::vector<int> px;
    px.reserve((size_t)W * H / std::max(1, c->n_shards) + T * T);
    for (int t = 0; t < tx * ty; ++t) {
        if (t % c->n_shards != c->shard_id) continue;
        int x0 = (t % tx) * T, y0 = (t / tx) * T;
        for (int my = 0; my < T; my += 8)
            for (int mx = 0; mx < T; mx += 8)
                for (int yy = 0; yy < 8; ++yy)
                    for (int xx = 0; xx < 8; ++xx) {
                        int x = x0 + mx + xx, y = y0 + my + yy;
                        if (mx + xx < T && my + yy < T && x < W && y < H) px.push_back(y * W + x);
                    }
    }
    if (c->d_work) hipFree(c->d_work);
    c->d_work = nullptr;
    HIPCHK(c, dalloc(&c->d_work, px.size()));
    HIPCHK(c, hipMemcpy(c->d_work, px.data(), px.size() * sizeof(int), hipMemcpyHostToDevice));
    c->n_work = (int)px.size();
    c->work_dirty = false;
    ++c->work_epoch;
    return RT_OK;
}

// Sampling.h:781-807 Continuous_Inversion_Sampler table (Riemann sum, renormalised, last entry 1) and the
// filters' 1-D factors (filters.h:101-107 Gaussian with helpers.h:221-225, 228-231 Lanczos with 236-251);
// powf(v, 2) is written v * v.
template <class F>
void inversion_table(F pdf, float a, float b, int N, std::vector<float>& cdf) {
    cdf.assign(N + 1, 0.0f);
    float delta_x = (b - a) / (float)N;
    float sum = 0;
    for (int n = 1; n < N + 1; n++) {
        float x = a + delta_x * n;
        float current_x = x < a ? a : (b < x ? b : x);
        sum += delta_x * pdf(current_x);
        cdf[n] = sum;
    }
    float scaling_term = 1.0f / cdf[N];
    for (int n = 1; n < N; n++) cdf[n] *= scaling_term;
    cdf[N] = 1.0f;
}
inline float gaussian_f(float x, float mu, float sigma) {
    const float Pi = 3.14159265358979323846f;
    float v = x - mu;
    return 1.0f / std::sqrt(2 * Pi * sigma * sigma) * std::exp(-(v * v) / (2 * sigma * sigma));
}
inline float sinx_over_x(float x) {
    if (1 - x * x == 1) return 1;
    return std::sin(x) / x;
}
inline float windowed_sinc(float x, float radius, float tau) {
    const float Pi = 3.14159265358979323846f;
    if (std::fabs(x) > radius) return 0;
    return sinx_over_x(Pi * x) * sinx_over_x(Pi * (x / tau));
}
int build_filter_tables(const rt_film_desc& d, std::vector<float>& tx, std::vector<float>& ty) {
    float rx = d.filter_radius[0], ry = d.filter_radius[1];
    if (d.filter == RT_FILTER_GAUSSIAN) {
        float sigma = d.filter_param > 0 ? d.filter_param : 0.5f;
        float ex = gaussian_f(rx, 0, sigma), ey = gaussian_f(ry, 0, sigma);
        inversion_table([&](float x) { return std::max<float>(0, gaussian_f(x, 0, sigma) - ex); }, -rx, rx, 10000, tx);
        inversion_table([&](float y) { return std::max<float>(0, gaussian_f(y, 0, sigma) - ey); }, -ry, ry, 10000, ty);
        return 10000;
    }
    float tau = d.filter_param > 0 ? d.filter_param : 3.f;
    inversion_table([&](float x) { return windowed_sinc(x, rx, tau); }, -rx, rx, 2000, tx);
    inversion_table([&](float y) { return windowed_sinc(y, ry, tau); }, -ry, ry, 2000, ty);
    return 2000;
}

DevCamera dev_camera(const rt_camera_desc& d) {
    DevCamera c;
    std::memcpy(c.r2c, d.raster_to_camera, 64);
    std::memcpy(c.c2w, d.camera_to_world, 64);
    c.lens_radius = d.lens_radius;
    c.focal_distance = d.focal_distance;
    c.type = d.type;
    std::memcpy(c.r2s, d.raster_to_screen, 64);
    c.pinhole_depth = d.pinhole_depth;
    c.thin_focal = d.thin_focal;
    c.thin_aperture = d.thin_aperture_diameter;
    c.sensor_depth = d.sensor_depth;
    return c;
}
// Sobol generator matrices (32 dimensions, Joe-Kuo new-joe-kuo-6.21201 direction numbers; dimension 0 = van der
// Corput) and SobolIntervalToIndex's tables for a resolution exponent m (the reference's VdCSobolMatrices /
// VdCSobolMatricesInv, HelperFunctions.h:212-470, derived here by inverting the 2m x 2m GF(2) pixel map).
void sobol_tables(int m, std::vector<uint32_t>& mats, std::vector<uint64_t>& fwd, std::vector<uint64_t>& inv) {
    static const int dirs[31][9] = {
        {1, 0, 1}, {2, 1, 1, 3}, {3, 1, 1, 3, 1}, {3, 2, 1, 1, 1}, {4, 1, 1, 1, 3, 3}, {4, 4, 1, 3, 5, 13},
        {5, 2, 1, 1, 5, 5, 17}, {5, 4, 1, 1, 5, 5, 5}, {5, 7, 1, 1, 7, 11, 19}, {5, 11, 1, 1, 5, 1, 1},
        {5, 13, 1, 1, 1, 3, 11}, {5, 14, 1, 3, 5, 5, 31}, {6, 1, 1, 3, 3, 9, 7, 49}, {6, 13, 1, 1, 1, 15, 21, 21},
        {6, 16, 1, 3, 1, 13, 27, 49}, {6, 19, 1, 1, 1, 15, 7, 5}, {6, 22, 1, 3, 1, 15, 13, 25},
        {6, 25, 1, 1, 5, 5, 19, 61}, {7, 1, 1, 3, 7, 11, 23, 15, 103}, {7, 4, 1, 3, 7, 13, 13, 15, 69},
        {7, 7, 1, 1, 3, 13, 7, 35, 63}, {7, 8, 1, 3, 5, 9, 1, 25, 53}, {7, 14, 1, 3, 1, 13, 9, 35, 107},
        {7, 19, 1, 3, 1, 5, 27, 61, 31}, {7, 21, 1, 1, 5, 11, 19, 41, 61}, {7, 28, 1, 3, 5, 3, 3, 13, 69},
        {7, 31, 1, 1, 7, 13, 1, 19, 1}, {7, 32, 1, 3, 7, 5, 13, 19, 59}, {7, 37, 1, 1, 3, 9, 25, 29, 41},
        {7, 41, 1, 3, 5, 13, 23, 1, 55}, {7, 42, 1, 3, 7, 3, 13, 59, 17}};
    const int S = kSobolMatrixSize;
    mats.assign((size_t)kSobolDims * S, 0u);
    for (int j = 0; j < 32; ++j) mats[j] = 1u << (31 - j);
    for (int d = 1; d < kSobolDims; ++d) {
        int s = dirs[d - 1][0], a = dirs[d - 1][1];
        uint64_t dn[kSobolMatrixSize];
        for (int i = 0; i < s; ++i) dn[i] = (uint64_t)dirs[d - 1][2 + i];
        for (int i = s; i < S; ++i) {  // m_i = 2^s m_{i-s} ^ m_{i-s} ^ sum_k a_k 2^k m_{i-k}
            uint64_t v = dn[i - s] ^ (dn[i - s] << s);
            for (int k = 1; k < s; ++k)
                if ((a >> (s - 1 - k)) & 1) v ^= dn[i - k] << k;
            dn[i] = v;
        }
        for (int j = 0; j < S; ++j) mats[(size_t)d * S + j] = (uint32_t)((dn[j] << (63 - j)) >> 32);
    }
    fwd.assign(S, 0);
    inv.assign(S, 0);
    if (m == 0) return;
    const int n = 2 * m;
    auto col = [&](int j) { return ((uint64_t)(mats[j] >> (32 - m)) << m) | (uint64_t)(mats[S + j] >> (32 - m)); };
    for (int c = 0; c + n < S; ++c) fwd[c] = col(n + c);
    uint64_t rows[32], id[32];
    for (int r = 0; r < n; ++r) {
        rows[r] = 0;
        for (int j = 0; j < n; ++j) rows[r] |= ((col(j) >> r) & 1ull) << j;
        id[r] = 1ull << r;
    }
    for (int c = 0; c < n; ++c) {
        int p = c;
        while (!((rows[p] >> c) & 1)) ++p;
        std::swap(rows[p], rows[c]);
        std::swap(id[p], id[c]);
        for (int r = 0; r < n; ++r)
            if (r != c && ((rows[r] >> c) & 1)) { rows[r] ^= rows[c]; id[r] ^= id[c]; }
    }
    for (int c = 0; c < n; ++c)  // column c of M^-1: index bits set by pixel bit c
        for (int r = 0; r < n; ++r) inv[c] |= ((id[r] >> c) & 1ull) << r;
}

DevSampler dev_sampler(const rt_ctx* c) {
    const rt_sampler_desc& d = c->smp;
    DevSampler s{};
    s.kind = d.kind; s.xs = d.x_samples; s.ys = d.y_samples; s.jitter = d.jitter; s.seed = d.seed;
    s.spp = d.kind == RT_SAMPLER_STRATIFIED ? d.x_samples * d.y_samples : d.x_samples;
    s.randomize = d.randomize;
    s.sobol_m = c->sobol_m;
    s.scale = 1 << c->sobol_m;
    s.sobol_mats = c->d_sobol_mats;
    s.sobol_fwd = c->d_sobol_fwd;
    s.sobol_inv = c->d_sobol_fwd ? c->d_sobol_fwd + kSobolMatrixSize : nullptr;
    auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
    if (s.kind == RT_SAMPLER_STRATIFIED && pow2(s.xs) && pow2(s.ys)) {
        s.p2 = 1;
        while ((1 << s.lg_xs) < s.xs) ++s.lg_xs;
        s.inv_xs = 1.0f / (float)s.xs;   // exact: powers of two
        s.inv_ys = 1.0f / (float)s.ys;
        s.inv_spp = 1.0f / (float)s.spp;
    }
    return s;
}

// sample ids of a batch starting at sample index b0 (s = i n_pixels + j)
SampleIds sample_ids(const rt_ctx* c, int b0) {
    SampleIds ids{c->d_work, c->n_work, b0, nullptr, nullptr};
    ids.np_div = make_intdiv((uint32_t)c->n_work);
    return ids;
}

// Sobol tables on the device for the current film (scale = RoundUpPow2(max(res)), samplers.h:243)
int ensure_sobol(rt_ctx* c) {
    if (c->smp.kind != RT_SAMPLER_SOBOL) return RT_OK;
    int v = std::max(c->film.res_x, c->film.res_y) - 1;
    v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    int m = (int)std::log2((float)(v + 1));
    if (m > 16) return fail(c, RT_E_LIMIT, "Sobol sampler supports film resolutions up to 65536");
    if (c->d_sobol_mats && c->sobol_m == m) return RT_OK;
    std::vector<uint32_t> mats;
    std::vector<uint64_t> fwd, inv;
    sobol_tables(m, mats, fwd, inv);
    if (!c->d_sobol_mats) {
        HIPCHK(c, hipMalloc(&c->d_sobol_mats, mats.size() * 4));
        HIPCHK(c, hipMalloc(&c->d_sobol_fwd, 2 * kSobolMatrixSize * 8));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(c->d_sobol_mats, mats.data(), mats.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_sobol_fwd, fwd.data(), kSobolMatrixSize * 8, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_sobol_fwd + kSobolMatrixSize, inv.data(), kSobolMatrixSize * 8, hipMemcpyHostToDevice));
    c->sobol_m = m;
    return RT_OK;
}
DevFilm dev_film(const rt_ctx* c) {
    const rt_film_desc& d = c->film;
    DevFilm f;
    f.res_x = d.res_x; f.res_y = d.res_y; f.filter = d.filter;
    f.rx = d.filter_radius[0]; f.ry = d.filter_radius[1]; f.imaging_ratio = d.imaging_ratio;
    f.cdf_x = c->d_cdf;
    f.cdf_y = c->d_cdf ? c->d_cdf + (c->cdf_n + 1) : nullptr;
    f.cdf_n = c->cdf_n;
    f.rx_div = make_intdiv((uint32_t)d.res_x);
    f.y_int = c->film_y_int;
    return f;
}

ShadeRefIO shade_ref_io(rt_ctx* c) {
    ShadeRefIO io{};
    io.rsh = 1;  // the workspace's interleaved rays
    float a = c->integ.albedo_rgb[0];
    io.albedo_c2 = (a - .5f) / std::sqrt(a * (1 - a));  // color.cpp:35-37
    float g = 1.0f / (2.0f * 1.0f);                      // RGBIlluminant(1,1,1): scale = 2*max = 2, rgb/scale = .5
    io.illum_c2 = (g - .5f) / std::sqrt(g * (1 - g));
    io.illum_scale = 2.0f;
    return io;
}

int check_ready(rt_ctx* c) {
    if (!c) return RT_E_ARG;
    if (!c->have_scene || !c->have_cam || !c->have_smp || !c->have_film || !c->have_integ)
        return fail(c, RT_E_STATE, "scene, camera, sampler, film and integrator must be set before rendering");
    // The multi-level BVH decides rays whose origin lies within oguard = 8 M of the scene's vertices' extent M
    // (scene_bvh); a camera eye farther out sends every camera ray to the exact octree BFS.  Correct, but a large
    // performance cliff that only the fallback counter shows: say so once per context.
    if (c->dsc.oguard > 0.f && !c->warned_eye) {
        const float* t = c->cam.camera_to_world + 12;  // column-major: the translation column
        if (std::max(std::fabs(t[0]), std::max(std::fabs(t[1]), std::fabs(t[2]))) > c->dsc.oguard) {
            std::fprintf(stderr, "rtmi355x: the camera eye lies beyond the BVH's origin guard (8x the scene extent): "
                                 "every camera ray takes the exact octree BFS (slow, still exact)\n");
            c->warned_eye = true;
        }
    }
    return RT_OK;
}

// Calls on a context may use different streams (rt_render_pass on the context's stream, rt_render_pass_device on the
// caller's, the debug entry points): each waits for the previous call's work, which shares the lane-0 buffers.
int order_after_previous(rt_ctx* c, hipStream_t st) {
    if (!c->done) HIPCHK(c, hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    else HIPCHK(c, hipStreamWaitEvent(st, c->done, 0));
    return RT_OK;
}
int mark_done(rt_ctx* c, hipStream_t st) {
    HIPCHK(c, hipEventRecord(c->done, st));
    return RT_OK;
}

int render_device_body(rt_ctx* c, int ib, int ie, float4* film, hipStream_t st);
// one render pass over [ib, ie) into the device film
int render_device(rt_ctx* c, int ib, int ie, float4* film, hipStream_t st) {
    int rc = check_ready(c);
    if (rc) return rc;
    if ((rc = order_after_previous(c, st))) return rc;
    rc = render_device_body(c, ib, ie, film, st);
    int rc2 = mark_done(c, st);
    return rc ? rc : rc2;
}

int render_device_body(rt_ctx* c, int ib, int ie, float4* film, hipStream_t st) {
    int rc;
    if (ib < 0 || ie < ib) return fail(c, RT_E_ARG, "invalid index range");
    if ((rc = ensure_sobol(c))) return rc;
    DevSampler smp = dev_sampler(c);
    if (c->smp.kind == RT_SAMPLER_STRATIFIED && !c->smp.jitter && ie > smp.spp)
        return fail(c, RT_E_ARG, "StratifiedSampler without jitter supports indices < SamplesPerPixel (samplers.h:83-87)");
    if ((rc = build_work(c))) return rc;
    if (ie == ib || c->n_work == 0) return RT_OK;
    bool path = c->integ.kind == RT_INTEGRATOR_PATH || c->integ.kind == RT_INTEGRATOR_PATH_MIS;
    c->dsc.mis = c->integ.kind == RT_INTEGRATOR_PATH_MIS;
    c->dsc.full = c->scene_full || c->dsc.mis;
    // samples per path batch: 16 Mi on a single-leaf octree (8 Mi: Cornell 1874 -> 1827; flat above 16 Mi, r06_ab7),
    // 32 Mi on multi-level ones, whose fewer, fuller launches keep more rays in every wave's reach (16 -> 32 Mi: CFG3
    // +2.5 %, CFG4 +3.5 %, flat above, r06_ab23/24)
    const size_t target = c->batch_samples ? c->batch_samples : (size_t)(c->dsc.qcap == 1 ? 16 : 32) << 20;
    int B = (int)std::max<size_t>(1, target / (size_t)c->n_work);
    B = std::min(B, ie - ib);
    size_t nmax = (size_t)B * c->n_work;
    // queue / hit capacity: the shards of the largest batch (>= nmax); single-leaf scenes use one shard
    const int nsh = c->dsc.qcap == 1 ? 1 : kShards;
    const size_t ncap = (size_t)nsh * (size_t)shard_stride((int)nmax, nsh);
    DevCamera cam = dev_camera(c->cam);
    DevFilm fd = dev_film(c);
    if (!path) {
        Work& w = c->ws[0];
        if ((rc = ensure_workspace(c, w, ncap, false))) return rc;
        for (int b0 = ib; b0 < ie; b0 += B) {
            int nIdx = std::min(B, ie - b0);
            int nS = nIdx * c->n_work;
            SampleIds ids = sample_ids(c, b0);
            GenOut go{w.rayO, w.rayD, w.lamA, w.lamB, w.pdfA, w.pdfB, RecView{nullptr, 0, 0}, 0, 1};
            hipEvent_t e0 = ev_start(c, st);
            HIPCHK(c, launch_generate(st, c->grid, nS, ids, cam, smp, fd, go));
            ev_mark(c, st, ST_GEN, e0);
            TraceIO tio{w.rayO, w.rayD, QueueView{nullptr, shard_stride(nS, nsh), nS, nsh}, c->cull ? 1 : 0, w.hitB, w.hitPrim,
                        nullptr, 1};
            e0 = ev_start(c, st);
            HIPCHK(c, launch_trace_closest(st, 0, c->dsc.qcap, lane_scene(c, w), tio, c->d_ctr));
            ev_mark(c, st, ST_TRACE, e0);
            ShadeRefIO sio = shade_ref_io(c);
            sio.work_pixels = c->d_work; sio.n_pixels = c->n_work; sio.n_index = nIdx;
            sio.rayD = w.rayD; sio.lamA = w.lamA; sio.lamB = w.lamB; sio.pdfA = w.pdfA; sio.pdfB = w.pdfB;
            sio.hitB = w.hitB; sio.hitPrim = w.hitPrim; sio.film = film;
            e0 = ev_start(c, st);
            HIPCHK(c, launch_ref_shade_film(st, 0, c->dsc, c->d_spec, fd, sio, c->d_ctr));
            ev_mark(c, st, ST_FILM, e0);
        }
        return RT_OK;
    }

    // ---- path mode: up to c->lanes batches in flight, batch k on lane k mod lanes (lane 0 = the caller's stream).
    // Within a lane everything is stream-ordered; across lanes only the film kernels are chained (batch k's film
    // after batch k-1's), so every pixel still adds its sample indices in increasing order.
    const int nbatch = (ie - ib + B - 1) / B;
    const int lanes = std::max(1, std::min(std::min(c->lanes, kLanes), nbatch));
    // multi-level octrees: coherence-sort each bounce's rays (rt_sort.hip); on the single-leaf Cornell box the sort
    // costs more than it saves (1110 -> 720 Msamples/s)
    const bool sort_rays = c->dsc.qcap != 1 && c->sort_rays;
    for (int l = 0; l < lanes; ++l) {
        if ((rc = ensure_workspace(c, c->ws[l], ncap, true))) return rc;
        if (sort_rays && (rc = ensure_sort_workspace(c, c->ws[l], ncap))) return rc;
        if (c->dsc.qcap != 1 && (rc = ensure_trace_fallback(c, c->ws[l], ncap))) return rc;
    }
    // Cornell-like single-leaf scenes cost the same per ray: static chunks on a resident grid beat tickets there
    // (A/B 1229 vs 1106-1158 Msamples/s); multi-level octrees vary per ray by 100x: tickets (CFG3 71 -> 96)
    const bool dyn = c->dsc.qcap != 1;
    // k_generate stores no β = 1 / L = 0 / pdf streams: depth 0 starts from them in registers and the film recomputes
    // the pdf (simple path: +4.5 %).  1: the simple path (the host derives each depth's sampler dimension); 2: mixed
    // scenes, whose slots keep their dimension, prevPdf and TerminateSecondary flag in R_MISC (CFG4: k_generate
    // writes 96 instead of 192 B per sample)
    const int lean = c->dsc.full ? 2 : 1;
    // multi-level simple scenes: the NEE shadow rays the BVH alone cannot decide (or, with RTMI_SHADOW_QUEUE=1,
    // all of them) are queued and traced exactly by their own kernel
    const bool shq = c->dsc.qcap != 1 && !c->dsc.full;
    if (shq)
        for (int l = 0; l < lanes; ++l)
            if ((rc = ensure_shadow_workspace(c, c->ws[l], ncap))) return rc;
    // mixed scenes: NEE deferred to k_path_nee (one record per slot, one queue entry per Lambert vertex)
    const bool nee = c->dsc.full && c->dsc.n_lights > 0;
    if (nee)
        for (int l = 0; l < lanes; ++l)
            if ((rc = ensure_nee_workspace(c, c->ws[l], nmax * (size_t)nee_stride(c->dsc.n_lights),
                                           (3 + kMatClasses) * (size_t)ncap)))
                return rc;  // (the NEE queue, the fallback list, the NEE sort keys: rt_internal.h NeeIO; the
                            // material bins' index lists: TraceIO bin_idx)
    // mixed multi-level scenes: the trace kernel bins the hits by material class and each class is shaded by a kernel
    // holding only its materials' code (k_path_shade_full<Q, 1 / 2>)
    const bool bins = nee && c->dsc.qcap != 1 && c->mat_bins;
    // Concurrent lanes share the CUs.  Each launch still asks for every resident block (grid_div 1): the dispatcher
    // hands blocks to whichever lane's kernel has them pending, so a VALU-bound trace and an HBM-bound shade of the
    // other lane end up co-resident (Cornell A/B: 1 lane 1217, 2 lanes with half grids 1422, with full grids 1500)
    const int grid = c->grid;
    auto lstream = [&](int l) { return l == 0 ? st : c->ws[l].stream; };
    if (lanes > 1) {  // lanes 1.. start after the caller's earlier work on st
        HIPCHK(c, hipEventRecord(c->ws[0].film_done, st));
        for (int l = 1; l < lanes; ++l) HIPCHK(c, hipStreamWaitEvent(c->ws[l].stream, c->ws[0].film_done, 0));
    }
    const size_t qs = ncap;  // one queue (nsh shards of stride Sq[lane])
    // slot state layout (rt_internal.h RecView): records for multi-level scenes (sorted, scattered slots), SoA for
    // single-leaf ones (slots stay in queue order)
    const bool records = c->dsc.qcap != 1;
    const size_t rec_fs = records ? 1 : nmax;
    const unsigned rec_ss = records ? (unsigned)kRecF4 : 1u;
    const int rec_rng8 = !records && lean == 1 ? 1 : 0;  // SoA simple path: dense 8-byte PCG states
    int last_film = -1;      // lane of the most recent film launch
    for (int g0 = ib; g0 < ie; g0 += B * lanes) {
        int nIdx[kLanes] = {0}, cur[kLanes] = {0}, nSq[kLanes] = {0}, Sq[kLanes] = {0};
        for (int l = 0; l < lanes; ++l) {
            int b0 = g0 + l * B;
            if (b0 >= ie) break;
            Work& w = c->ws[l];
            hipStream_t s = lstream(l);
            const RecView rv{w.rec, rec_fs, rec_ss, rec_rng8};
            nIdx[l] = std::min(B, ie - b0);
            int nS = nIdx[l] * c->n_work;
            nSq[l] = nS;
            Sq[l] = shard_stride(nS, nsh);  // every queue of this batch: shard j at [j S, j S + len_j)
            SampleIds ids = sample_ids(c, b0);
            GenOut go{w.rayO, w.rayD, nullptr, nullptr, w.pdfA, w.pdfB, rv, lean, 1};
            // camera rays fill queue 0 densely (positions 0..nS-1: QueueView without lengths); both counter regions
            // start at zero: k_generate zeroes them (a memset launch here waited for the other lane's resident blocks
            // in two-lane mode, r05 kernel traces)
            go.zero = w.d_qcount;
            hipEvent_t e0 = ev_start(c, s);
            HIPCHK(c, launch_generate(s, grid, nS, ids, cam, smp, fd, go));
            ev_mark(c, s, ST_GEN, e0);
        }
        for (int depth = 0; depth <= c->integ.max_depth; ++depth) {
            // the last trace can only add emitter hits, which count only after specular bounces or with MIS
            if (depth == c->integ.max_depth && depth > 0 && !c->dsc.full) break;
            for (int l = 0; l < lanes && nIdx[l] > 0; ++l) {
                Work& w = c->ws[l];
                hipStream_t s = lstream(l);
                const RecView rv{w.rec, rec_fs, rec_ss, rec_rng8};
                SampleIds ids = sample_ids(c, g0 + l * B);
                int nxt = cur[l] ^ 1;
                const float4* cO = w.rayO + 2 * (size_t)cur[l] * qs;
                const float4* cD = cO + 1;
                int* qc_cur = w.d_qcount + kQRegion * cur[l];
                int* qc_nxt = w.d_qcount + kQRegion * nxt;
                // the next queue's length and the chunk tickets its trace and shade launches will use start at zero:
                // depth 0 (k_generate zeroed both regions) / the trace kernel zeroes it (below), except before the
                // emitter filter, which appends to it ahead of the trace
                const bool efilter0 = c->emit_filter && c->dsc.full && depth == c->integ.max_depth && depth > 0 &&
                                      c->dsc.n_emit_tris >= 0;
                if (efilter0) HIPCHK(c, hipMemsetAsync(qc_nxt, 0, kQRegion * sizeof(int), s));
                hipEvent_t e0;
                // multi-level octrees: bounce rays sorted by (octant, direction cell, origin Morton code) before
                // the trace.  The queue length is read back so only live rays are sorted (sorting the capacity with
                // padded keys instead, without the host read: -0.6 %); the other lane keeps the GPU busy meanwhile.
                QueueView qv = depth == 0 ? QueueView{nullptr, Sq[l], nSq[l], nsh}
                                          : QueueView{qc_cur + kQLen, Sq[l], 0, nsh};
                const DevScene dsl = lane_scene(c, w);
                // the last depth of a mixed scene: only emitter hits still add to L, so the rays that hit no emissive
                // surface are dropped first (k_emitter_filter, EmitIO) into the free next queue, whose rays the trace
                // and shade kernels then take (the shade appends nothing at this depth); no coherence sort
                const bool efilter = c->emit_filter && c->dsc.full && depth == c->integ.max_depth && depth > 0 &&
                                     c->dsc.n_emit_tris >= 0;
                if (efilter) {
                    const EmitIO eio{qv, cO, w.rayO + 2 * (size_t)nxt * qs, qc_nxt + kQLen};
                    e0 = ev_start(c, s);
                    HIPCHK(c, launch_emitter_filter(s, grid, dsl, eio));
                    ev_mark(c, s, ST_FILTER, e0);
                    cO = eio.nO;
                    cD = cO + 1;
                    qv = QueueView{qc_nxt + kQLen, Sq[l], 0, nsh};
                }
                TraceIO tio{cO, cD, qv, 0, w.hitB, w.hitPrim, dyn ? qc_cur + kQTraceTicket : nullptr, 1};
                if (depth > 0 && !efilter) tio.zero = qc_nxt;
                if (c->dsc.qcap != 1) {  // ambiguous rays listed for k_trace_fallback (the trace holds no BFS)
                    tio.fb_pos = w.tfb;
                    tio.fb_len = qc_cur + kQTraceFallback;
                }
                BinIO bio{qv, w.hitPrim, {w.neeSlot + 3 * ncap, w.neeSlot + 4 * ncap}, qc_cur + kQBinLen};
                if (depth == 0) { bio.rayO = cO; bio.rec = rv; }  // lean depth 0: the misses' L = 0 (BinIO)
                static_assert(kMatClasses == 2, "bin index lists");
                if (sort_rays && depth > 0 && !efilter) {  // the device reads the queue length itself: no host read
                    SortRaysIO so{w.sQKey, w.sS, w.sKeys, w.sKeysAlt, w.sVals, w.sValsAlt, w.sTemp,
                                  c->sort_dir_bits, c->sort_org_bits, qc_cur + kQLen, Sq[l]};
                    e0 = ev_start(c, s);
                    HIPCHK(c, launch_sort_rays(s, so));
                    ev_mark(c, s, ST_SORT, e0);
                    tio.perm = w.sS;  // the trace kernel gathers the sorted rays into the side queue
                    tio.so = w.sO;
                    cO = w.sO; cD = w.sD;
                }
                e0 = ev_start(c, s);
                HIPCHK(c, launch_trace_closest(s, grid, c->dsc.qcap, dsl, tio, c->d_ctr));
                // (an ambiguous ray is listed only if the cooperative BFS's FIFO overflows, which the octree's exact
                // queue bound excludes when coop_ok: then no launch, which in two-lane mode would wait for the other
                // lane's resident blocks, r05 kernel traces: 1.28 ms per bounce)
                if (tio.fb_pos && !c->dsc.coop_ok)
                    HIPCHK(c, launch_trace_fallback(s, grid, c->dsc.qcap, dsl, tio, c->d_ctr));
                ev_mark(c, s, ST_TRACE, e0);
                PathIO pio{};
                pio.lean = lean;
                pio.rayO = cO; pio.rayD = cD; pio.q = qv;
                pio.hitB = w.hitB; pio.hitPrim = w.hitPrim;
                pio.nO = w.rayO + 2 * (size_t)nxt * qs; pio.nD = pio.nO + 1;
                pio.nCount = qc_nxt + kQLen;
                pio.rec = rv; pio.pdfA = w.pdfA; pio.pdfB = w.pdfB;
                pio.depth = depth; pio.max_depth = c->integ.max_depth;
                pio.dim = -1;
                if (lean == 1) {
                    pio.dim = dim_after_camera(smp, cam);
                    for (int d = 0; d < depth; ++d) pio.dim = dim_get2d(smp, dim_get2d(smp, pio.dim));
                }
                pio.ticket = dyn ? qc_cur + kQShadeTicket : nullptr;
                if (sort_rays && depth < c->integ.max_depth) {  // keys of the rays this shade appends (next sort)
                    pio.nkey.key = w.sQKey;
                    pio.nkey.lo = c->sort_lo;
                    pio.nkey.scale = c->sort_scale;
                    pio.nkey.dir_bits = c->sort_dir_bits;
                    pio.nkey.org_bits = c->sort_org_bits;
                    pio.nkey.org_major = c->sort_org_major >= 0 ? c->sort_org_major : (c->dsc.full ? 0 : 1);
                }
                ShadowQueueIO sqio{};
                if (shq) {  // this queue's region holds the shadow-queue length and ticket (zeroed with it)
                    sqio.shO = w.shO; sqio.shD = w.shD; sqio.shLA = w.shLA; sqio.shLB = w.shLB;
                    sqio.shCount = qc_cur + kQShadowLen;
                    sqio.shTicket = qc_cur + kQShadowTicket;
                    sqio.defer = c->shadow_queue ? 0 : 1;
                }
                NeeIO nio{};
                const bool sort_nee = nee && sort_rays && c->sort_nee;
                unsigned* nee_key = reinterpret_cast<unsigned*>(w.neeSlot + 2 * ncap);
                if (nee)
                    nio = NeeIO{w.neeRec, w.neeSlot, qc_cur + kQShadowLen, qc_cur + kQShadowTicket, w.neeSlot + ncap,
                                qc_cur + kQNeeFallback, sort_nee ? nee_key : nullptr, c->sort_lo, c->sort_scale,
                                c->sort_nee_bits};
                e0 = ev_start(c, s);
                if (bins) {  // the hits binned by material, then one kernel per bin over its index list
                    HIPCHK(c, launch_bin_materials(s, grid, dsl, bio));
                    for (int cl = 0; cl < kMatClasses; ++cl) {
                        PathIO bp = pio;
                        bp.q = QueueView{qc_cur + kQBinLen + cl * kShards * kQStride, Sq[l], 0, nsh};
                        bp.ticket = qc_cur + kQBinTicket + cl * kShards * kQStride;
                        bp.bin_idx = bio.idx[cl];
                        HIPCHK(c, launch_path_shade(s, grid, c->dsc.qcap, dsl, c->d_spec, smp, fd, ids, bp, c->d_ctr,
                                                    sqio, nio, 1 + cl));
                    }
                } else {
                    HIPCHK(c, launch_path_shade(s, grid, c->dsc.qcap, dsl, c->d_spec, smp, fd, ids, pio, c->d_ctr, sqio,
                                                nio));
                }
                ev_mark(c, s, ST_SHADE, e0);
                if (sort_nee) {  // NEE vertices in Morton order of their shading points (no host round trip)
                    SortNeeIO so{w.neeSlot, qc_cur + kQShadowLen, Sq[l], nee_key, w.sKeys, w.sKeysAlt, w.sVals,
                                 w.sValsAlt, w.sTemp, c->sort_nee_bits};
                    e0 = ev_start(c, s);
                    HIPCHK(c, launch_sort_nee(s, so));
                    ev_mark(c, s, ST_SORT, e0);
                }
                if (nee) {  // this bounce's shadow rays, before the next bounce reads L
                    e0 = ev_start(c, s);
                    HIPCHK(c, launch_path_nee(s, grid, c->dsc.qcap, dsl, c->d_spec, pio, nio, c->d_ctr));
                    // (no fallback launch when k_path_nee resolves its undecided shadow rays itself, coop_ok)
                    if (c->dsc.qcap != 1 && !c->dsc.coop_ok)
                        HIPCHK(c, launch_path_nee_fallback(s, grid, c->dsc.qcap, dsl, c->d_spec, pio, nio, c->d_ctr));
                    ev_mark(c, s, ST_SHADOW, e0);
                }
                // (the deferred shadow rays are resolved in k_path_shade itself when coop_ok: no launch, which in
                // two-lane mode waits for the other lane's resident blocks, r05 kernel traces: 0.87 ms per bounce)
                if (shq && !(sqio.defer && c->dsc.coop_ok)) {
                    e0 = ev_start(c, s);
                    HIPCHK(c, launch_path_shadow(s, grid, c->dsc.qcap, c->shadow_dfs != 0, dsl, pio, sqio, c->d_ctr));
                    ev_mark(c, s, ST_SHADOW, e0);
                }
                cur[l] = nxt;
            }
        }
        for (int l = 0; l < lanes && nIdx[l] > 0; ++l) {
            Work& w = c->ws[l];
            hipStream_t s = lstream(l);
            const RecView rv{w.rec, rec_fs, rec_ss, rec_rng8};
            if (last_film >= 0 && last_film != l) HIPCHK(c, hipStreamWaitEvent(s, c->ws[last_film].film_done, 0));
            PathFilmIO fio{c->d_work, c->n_work, nIdx[l], rv, w.pdfA, w.pdfB, film};
            fio.lean = lean;
            hipEvent_t e0 = ev_start(c, s);
            HIPCHK(c, launch_path_film(s, 0, c->d_spec, fd, fio, c->d_ctr));
            ev_mark(c, s, ST_FILM, e0);
            HIPCHK(c, hipEventRecord(w.film_done, s));
            last_film = l;
        }
    }
    // the caller's stream resumes after every lane's last film
    for (int l = 1; l < lanes; ++l) HIPCHK(c, hipStreamWaitEvent(st, c->ws[l].film_done, 0));
    return RT_OK;
}

// ---------------------------------------------------------------------------------- PixelSensor (a18, a20)
// glm float order throughout: mat3 is column-major (m[col * 3 + row]); inverse = glm's cofactor form; products
// sum (a0 b0 + a1 b1) + a2 b2.
void inv3(const float* a, float* o) {
    auto m = [&](int col, int row) { return a[col * 3 + row]; };
    float ood = 1.0f / (+m(0, 0) * (m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2)) -
                        m(1, 0) * (m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2)) +
                        m(2, 0) * (m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2)));
    o[0] = +(m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2)) * ood;
    o[3] = -(m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2)) * ood;
    o[6] = +(m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1)) * ood;
    o[1] = -(m(0, 1) * m(2, 2) - m(2, 1) * m(0, 2)) * ood;
    o[4] = +(m(0, 0) * m(2, 2) - m(2, 0) * m(0, 2)) * ood;
    o[7] = -(m(0, 0) * m(2, 1) - m(2, 0) * m(0, 1)) * ood;
    o[2] = +(m(0, 1) * m(1, 2) - m(1, 1) * m(0, 2)) * ood;
    o[5] = -(m(0, 0) * m(1, 2) - m(1, 0) * m(0, 2)) * ood;
    o[8] = +(m(0, 0) * m(1, 1) - m(1, 0) * m(0, 1)) * ood;
}
void mul3(const float* A, const float* B, float* o) {
    for (int col = 0; col < 3; ++col)
        for (int r = 0; r < 3; ++r)
            o[col * 3 + r] = (A[0 * 3 + r] * B[col * 3 + 0] + A[1 * 3 + r] * B[col * 3 + 1]) + A[2 * 3 + r] * B[col * 3 + 2];
}

// Spectra::Init's named illuminants (spectrum.cpp:2620-2637): FromInterleaved(.., normalize = true)
PLS named_illuminant(const HostSpectra& hs, int which) {
    static const float* const tab[] = {rtdata::illum_d65, rtdata::illum_a, rtdata::illum_d50, rtdata::illum_f1,
                                       rtdata::illum_f2, rtdata::illum_f3, rtdata::illum_f4, rtdata::illum_f5,
                                       rtdata::illum_f6, rtdata::illum_f7, rtdata::illum_f8, rtdata::illum_f9,
                                       rtdata::illum_f10, rtdata::illum_f11, rtdata::illum_f12, rtdata::illum_aces_d60};
    static const int n[] = {rtdata::illum_d65_n, rtdata::illum_a_n, rtdata::illum_d50_n, rtdata::illum_f1_n,
                            rtdata::illum_f2_n, rtdata::illum_f3_n, rtdata::illum_f4_n, rtdata::illum_f5_n,
                            rtdata::illum_f6_n, rtdata::illum_f7_n, rtdata::illum_f8_n, rtdata::illum_f9_n,
                            rtdata::illum_f10_n, rtdata::illum_f11_n, rtdata::illum_f12_n, rtdata::illum_aces_d60_n};
    return hs.interleaved(tab[which], n[which], true);
}

// pixelsensor.h:104-117 ProjectReflectance: (b_i(λ) refl(λ)) illum(λ) summed over λ = 360..830 (float loop),
// divided by Σ b2(λ) illum(λ)
template <class R, class I, class B1, class B2, class B3>
F3 project_reflectance(const R& refl, const I& illum, const B1& b1, const B2& b2, const B3& b3) {
    float g = 0, r0 = 0, r1 = 0, r2 = 0;
    for (float l = 360; l <= 830; ++l) {
        g += b2.query(l) * illum.query(l);
        r0 += b1.query(l) * refl.query(l) * illum.query(l);
        r1 += b2.query(l) * refl.query(l) * illum.query(l);
        r2 += b3.query(l) * refl.query(l) * illum.query(l);
    }
    return F3{r0 / g, r1 / g, r2 / g};
}

// XYZFromSensorRGB (pixelsensor.h:37-79) and the sRGB RGBFromXYZ (colorspace.cpp:13-28) of a film description,
// plus the sensor's dense r/g/b curves.
void sensor_matrices(const HostSpectra& hs, int sensor, int illum_id, float* xyz_from_sensor, float* rgb_from_xyz,
                     DenseS bars[3]) {
    auto xyz_of = [&](const PLS& s) {  // SpectrumToXYZ
        float X = inner_product(hs.X, s), Y = inner_product(hs.Y, s), Z = inner_product(hs.Z, s);
        return F3{X / 106.856895f, Y / 106.856895f, Z / 106.856895f};
    };
    auto xy_of = [](F3 c) { return std::pair<float, float>{c.x / (c.x + c.y + c.z), c.y / (c.x + c.y + c.z)}; };
    auto xyY = [](float x, float y) { return y == 0 ? F3{0, 0, 0} : F3{x * 1.0f / y, 1.0f, (1 - x - y) * 1.0f / y}; };
    // sRGB (colorspace.cpp:91-106): primaries, white = the D65 illuminant's xy
    F3 W = xyz_of(hs.D65);
    auto w = xy_of(W);
    F3 R = xyY((float).64, (float).33), G = xyY((float).3, (float).6), Bp = xyY((float).15, (float).06);
    float rgb[9] = {R.x, R.y, R.z, G.x, G.y, G.z, Bp.x, Bp.y, Bp.z}, irgb[9];
    inv3(rgb, irgb);
    F3 Cw = m3v(irgb, W);
    float dg[9] = {Cw.x, 0, 0, 0, Cw.y, 0, 0, 0, Cw.z}, xyzFromRgb[9];
    mul3(rgb, dg, xyzFromRgb);
    inv3(xyzFromRgb, rgb_from_xyz);
    PLS illum = named_illuminant(hs, illum_id);
    if (sensor == RT_SENSOR_XYZ) {
        bars[0] = hs.X; bars[1] = hs.Y; bars[2] = hs.Z;
        // pixelsensor.h:70-79: WhiteBalance(SpectrumToXYZ(sensorIllum).xy, sRGB.w) (color.h:616-629, Bradford)
        float lmsFromXyz[9] = {(float)0.8951, (float)-0.7502, (float)0.0389, (float)0.2664, (float)1.7135,
                               (float)-0.0685, (float)-0.1614, (float)0.0367, (float)1.0296};
        float xyzFromLms[9] = {(float)0.986993, (float)0.432305, (float)-0.00852866, (float)-0.147054, (float)0.51836,
                               (float)0.0400428, (float)0.159963, (float)0.0492912, (float)0.968487};
        auto sw = xy_of(xyz_of(illum));
        F3 src = xyY(sw.first, sw.second), dst = xyY(w.first, w.second);
        F3 sl = m3v(lmsFromXyz, src), dl = m3v(lmsFromXyz, dst);
        float corr[9] = {dl.x / sl.x, 0, 0, 0, dl.y / sl.y, 0, 0, 0, dl.z / sl.z}, t1[9];
        mul3(xyzFromLms, corr, t1);
        mul3(t1, lmsFromXyz, xyz_from_sensor);
        return;
    }
    // camera curves: PiecewiseLinearSpectrum::FromInterleaved(.., false) sampled densely (pixelsensor.h:41)
    int cam = sensor - 1;
    for (int ch = 0; ch < 3; ++ch)
        bars[ch] = to_dense(hs.interleaved(rtdata::camera_curves[cam][ch], rtdata::camera_curves_n[cam][ch], false));
    float rgbCamera[24][3], xyzOutput[24][3];
    for (int i = 0; i < 24; ++i) {
        PLS sw = hs.interleaved(rtdata::swatches[i], rtdata::swatches_n[i], false);
        F3 c3 = project_reflectance(sw, illum, bars[0], bars[1], bars[2]);
        rgbCamera[i][0] = c3.x; rgbCamera[i][1] = c3.y; rgbCamera[i][2] = c3.z;
    }
    float sensorWhiteG = inner_product(illum, bars[1]);
    float sensorWhiteY = inner_product(illum, hs.Y);
    for (int i = 0; i < 24; ++i) {
        PLS sw = hs.interleaved(rtdata::swatches[i], rtdata::swatches_n[i], false);
        F3 x3 = project_reflectance(sw, hs.D65d, hs.X, hs.Y, hs.Z);  // outputColorSpace->illuminant (dense D65)
        float k = sensorWhiteY / sensorWhiteG;
        xyzOutput[i][0] = x3.x * k; xyzOutput[i][1] = x3.y * k; xyzOutput[i][2] = x3.z * k;
    }
    // helpers.h:258-272 LinearLeastSquares<3>: AtA[i][j] / AtB[i][j] are glm [column i][row j]
    float AtA[9] = {0}, AtB[9] = {0};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int r = 0; r < 24; ++r) {
                AtA[i * 3 + j] += rgbCamera[r][i] * rgbCamera[r][j];
                AtB[i * 3 + j] += rgbCamera[r][i] * xyzOutput[r][j];
            }
    float AtAi[9], P[9];
    inv3(AtA, AtAi);
    mul3(AtAi, AtB, P);
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) xyz_from_sensor[c * 3 + r] = P[r * 3 + c];  // glm::transpose
}

int setup_sensor(rt_ctx* c, const rt_film_desc& d) {
    DenseS bars[3];
    sensor_matrices(c->hs, d.sensor, d.sensor_illum, c->resolveA, c->resolveB, bars);
    float both[18];
    std::memcpy(both, c->resolveA, 36);
    std::memcpy(both + 9, c->resolveB, 36);
    char* base = (char*)c->d_spec;
    if (hipMemcpy(c->d_resolve, both, sizeof(both), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(base + offsetof(DevSpectra, SR), bars[0].v.data(), 4 * kSpecN, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(base + offsetof(DevSpectra, SG), bars[1].v.data(), 4 * kSpecN, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(base + offsetof(DevSpectra, SB), bars[2].v.data(), 4 * kSpecN, hipMemcpyHostToDevice) != hipSuccess)
        return fail(c, RT_E_HIP, "sensor upload");
    std::vector<float4> spk(kSpecN);
    for (int i = 0; i < kSpecN; ++i)
        spk[i] = make_float4(bars[0].v[i], bars[1].v[i], bars[2].v[i], c->hs.D65d.v[i]);
    if (hipMemcpy(base + offsetof(DevSpectra, SPK), spk.data(), sizeof(float4) * kSpecN, hipMemcpyHostToDevice) !=
        hipSuccess)
        return fail(c, RT_E_HIP, "sensor upload");
    return RT_OK;
}


// ---- multi-device pass (rt_options.n_devices > 1).  Device 0 packs each peer's owned pixels of the
// caller's film into that peer's exchange buffer; the peer copies them over xGMI, scatters them into its own film,
// renders its tiles (the same kernels, the same per-pixel index order), packs them and copies them back; device 0
// scatters them into the caller's film.  Pure copies: the film is bit-identical to a one-device render.
int peer_prepare(rt_ctx* c, size_t j) {
    rt_ctx* p = c->peers[j];
    rt_ctx::PeerLink& L = c->links[j];
    hipSetDevice(p->device);
    int rc = build_work(p);
    if (rc) return fail(c, rc, "device " + std::to_string(p->device) + ": " + p->err);
    size_t n = (size_t)p->film.res_x * p->film.res_y;
    if (p->film_cap < n) {
        if (p->d_film) hipFree(p->d_film);
        p->d_film = nullptr;
        HIPCHK(c, dalloc(&p->d_film, n));
        p->film_cap = n;
    }
    if (p->xfer_cap < (size_t)p->n_work) {
        if (p->xfer) hipFree(p->xfer);
        p->xfer = nullptr;
        HIPCHK(c, dalloc(&p->xfer, (size_t)p->n_work));
        p->xfer_cap = p->n_work;
    }
    hipSetDevice(c->device);
    if (L.epoch != p->work_epoch) {
        if (L.cap < (size_t)p->n_work) {
            if (L.work0) hipFree(L.work0);
            if (L.xfer0) hipFree(L.xfer0);
            L.work0 = nullptr;
            L.xfer0 = nullptr;
            HIPCHK(c, dalloc(&L.work0, (size_t)p->n_work));
            HIPCHK(c, dalloc(&L.xfer0, (size_t)p->n_work));
            L.cap = p->n_work;
        }
        HIPCHK(c, hipMemcpyPeer(L.work0, c->device, p->d_work, p->device, sizeof(int) * p->n_work));
        L.n = p->n_work;
        L.epoch = p->work_epoch;
    }
    return RT_OK;
}

// the peer's half of a pass, on its own stream (runs in its own host thread: multi-level octrees sort with a
// host round trip per bounce, which must not serialise the devices)
int peer_pass(rt_ctx* c, size_t j, int ib, int ie) {
    rt_ctx* p = c->peers[j];
    const rt_ctx::PeerLink& L = c->links[j];
    hipSetDevice(p->device);
    hipStream_t ps = p->stream;
    const size_t bytes = sizeof(float4) * L.n;
    HIPCHK(p, hipStreamWaitEvent(ps, c->gathered, 0));
    if (L.n) {
        HIPCHK(p, hipMemcpyPeerAsync(p->xfer, p->device, L.xfer0, c->device, bytes, ps));
        HIPCHK(p, launch_film_scatter(ps, L.n, p->d_work, p->xfer, p->d_film));
    }
    int rc = render_device(p, ib, ie, p->d_film, ps);
    if (rc) return rc;
    if (L.n) {
        HIPCHK(p, launch_film_gather(ps, L.n, p->d_work, p->d_film, p->xfer));
        HIPCHK(p, hipMemcpyPeerAsync(L.xfer0, c->device, p->xfer, p->device, bytes, ps));
    }
    HIPCHK(p, hipEventRecord(p->gathered, ps));
    return RT_OK;
}

int render_multi(rt_ctx* c, int ib, int ie, float4* film, hipStream_t st) {
    if (c->peers.empty()) return render_device(c, ib, ie, film, st);
    int rc = check_ready(c);
    if (rc) return rc;
    if (ib < 0 || ie < ib) return fail(c, RT_E_ARG, "invalid index range");
    for (size_t j = 0; j < c->peers.size(); ++j)
        if ((rc = peer_prepare(c, j))) return rc;
    hipSetDevice(c->device);
    for (const rt_ctx::PeerLink& L : c->links)
        if (L.n) HIPCHK(c, launch_film_gather(st, L.n, L.work0, film, L.xfer0));
    HIPCHK(c, hipEventRecord(c->gathered, st));
    std::vector<int> prc(c->peers.size(), RT_OK);
    std::vector<std::thread> th;
    th.reserve(c->peers.size());
    for (size_t j = 0; j < c->peers.size(); ++j) th.emplace_back([&, j] { prc[j] = peer_pass(c, j, ib, ie); });
    rc = render_device(c, ib, ie, film, st);
    for (std::thread& t : th) t.join();
    hipSetDevice(c->device);
    if (rc) return rc;
    for (size_t j = 0; j < c->peers.size(); ++j)
        if (prc[j]) return fail(c, prc[j], "device " + std::to_string(c->peers[j]->device) + ": " + c->peers[j]->err);
    for (size_t j = 0; j < c->peers.size(); ++j) {
        const rt_ctx::PeerLink& L = c->links[j];
        HIPCHK(c, hipStreamWaitEvent(st, c->peers[j]->gathered, 0));
        if (L.n) HIPCHK(c, launch_film_scatter(st, L.n, L.work0, L.xfer0, film));
    }
    return RT_OK;
}

}  // namespace

// =========================================================================================== C-ABI
extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

static void destroy_one(rt_ctx* c);

static int create_one(const rt_options* opt, rt_ctx** out) {
    if (!out) return RT_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return RT_E_NODEVICE;
    int dev = opt ? opt->device : 0;
    if (dev < 0 || dev >= ndev) return RT_E_ARG;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return RT_E_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RT_E_NODEVICE;
    rt_ctx* c = new rt_ctx();
    c->device = dev;
    c->octree_build = opt ? opt->octree_build : RT_OCTREE_BUILD_DEVICE;
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return RT_E_HIP;
    }
    c->grid = prop.multiProcessorCount * 8;  // persistent grid: 8 blocks of 256 per CU
    if (std::getenv("RTMI_NO_STAGE_EVENTS")) c->stage_events = false;
    if (const char* e = std::getenv("RTMI_LANES")) c->lanes = std::max(1, std::min(kLanes, std::atoi(e)));
    if (const char* e = std::getenv("RTMI_SHADOW_QUEUE")) c->shadow_queue = std::atoi(e);
    if (const char* e = std::getenv("RTMI_SHADOW_DFS")) c->shadow_dfs = std::atoi(e);
    if (const char* e = std::getenv("RTMI_SORT")) c->sort_rays = std::atoi(e);
    if (const char* e = std::getenv("RTMI_BVH_CI")) c->bvh_node_cost = (float)std::atof(e);
    if (const char* e = std::getenv("RTMI_BVH_LEAF")) c->bvh_max_leaf = std::max(1, std::min(15, std::atoi(e)));
    parse_bvh_any(c->bvh_any_cost, c->bvh_any_leaf);
    if (const char* e = std::getenv("RTMI_FORCE_AMB")) c->force_amb = std::max(-1, std::min(30, std::atoi(e)));
    if (const char* e = std::getenv("RTMI_COOP")) c->coop = std::atoi(e) != 0;
    if (const char* e = std::getenv("RTMI_MAT_BINS")) c->mat_bins = std::atoi(e);
    if (const char* e = std::getenv("RTMI_EMIT_FILTER")) c->emit_filter = std::atoi(e);
    if (const char* e = std::getenv("RTMI_DEBUG_PATH_KERNELS")) c->debug_path = std::atoi(e) != 0;
    if (const char* e = std::getenv("RTMI_SORT_BITS")) {
        int db = 3, ob = 4, om = -1;
        const int got = std::sscanf(e, "%d/%d/%d", &db, &ob, &om);
        // the key is 3 octant bits + 2 x db direction bits + 3 x ob origin bits in one u32, ob <= 9 (spread3_9)
        if (got >= 2 && db >= 0 && db <= 9 && ob >= 0 && ob <= 9 && 3 + 2 * db + 3 * ob <= 32) {
            c->sort_dir_bits = db;
            c->sort_org_bits = ob;
            if (got == 3) c->sort_org_major = om < 0 ? -1 : (om ? 1 : 0);
        }
    }
    if (const char* e = std::getenv("RTMI_SORT_NEE")) std::sscanf(e, "%d/%d", &c->sort_nee, &c->sort_nee_bits);
    c->sort_nee_bits = std::max(1, std::min(9, c->sort_nee_bits));
    if (const char* e = std::getenv("RTMI_BATCH_SAMPLES")) c->batch_samples = (size_t)std::max(0L, std::atol(e));
    c->hs.init();
    if (dalloc(&c->d_spec, 1) != hipSuccess || dalloc(&c->ws[0].d_qcount, 2 * kQRegion) != hipSuccess ||
        dalloc(&c->d_ctr, kCtrWords) != hipSuccess || dalloc(&c->d_resolve, 18) != hipSuccess) {
        destroy_one(c);
        return RT_E_OOM;
    }
    DevSpectra ds{};
    std::memcpy(ds.X, c->hs.X.v.data(), 4 * kSpecN);
    std::memcpy(ds.Y, c->hs.Y.v.data(), 4 * kSpecN);
    std::memcpy(ds.Z, c->hs.Z.v.data(), 4 * kSpecN);
    std::memcpy(ds.D65, c->hs.D65d.v.data(), 4 * kSpecN);
    ds.f1_n = (int)c->hs.F1.l.size();
    std::memcpy(ds.f1_lambda, c->hs.F1.l.data(), 4 * ds.f1_n);
    std::memcpy(ds.f1_value, c->hs.F1.v.data(), 4 * ds.f1_n);
    ds.bk7_n = (int)c->hs.BK7.l.size();
    std::memcpy(ds.bk7_lambda, c->hs.BK7.l.data(), 4 * ds.bk7_n);
    std::memcpy(ds.bk7_value, c->hs.BK7.v.data(), 4 * ds.bk7_n);
    hipMemcpy(c->d_spec, &ds, sizeof(ds), hipMemcpyHostToDevice);
    hipMemset(c->d_ctr, 0, sizeof(unsigned long long) * kCtrWords);
    {
        rt_film_desc fd{};  // XYZ sensor under D65 until rt_film_set says otherwise
        if (setup_sensor(c, fd) != RT_OK) {
            destroy_one(c);
            return RT_E_HIP;
        }
    }
    *out = c;
    return RT_OK;
}

static void destroy_one(rt_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    for (Work& w : c->ws)
        if (w.stream) hipStreamSynchronize(w.stream);
    harvest(c);
    for (hipEvent_t e : c->pool) hipEventDestroy(e);
    free_scene(c);
    free_workspace(c);
    for (Work& w : c->ws) {
        if (w.d_qcount) hipFree(w.d_qcount);
        if (w.film_done) hipEventDestroy(w.film_done);
        if (w.stream) hipStreamDestroy(w.stream);
    }
    void* ptrs[] = {c->d_spec, c->d_ctr, c->d_resolve, c->d_work, c->d_film, c->d_cdf, c->d_sobol_mats,
                    c->d_sobol_fwd};
    for (void* p : ptrs)
        if (p) hipFree(p);
    if (c->done) hipEventDestroy(c->done);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : "null context"; }

// World-space triangles of a (validated) scene: ObjectToRender * vec4(p,1) per vertex (= the per-test transform,
// Shapes.h:1117-1122), back-face flags (Shapes.h:1339-1380) and degenerate flags (Shapes.h:1131).
struct SceneWorld {
    std::vector<F3> wv, tri3;
    std::vector<uint8_t> back, degen;
};
static void scene_world(const rt_scene_desc* s, SceneWorld& w) {
    const int nt = s->n_triangles, nv = s->n_vertices;
    w.wv.resize(nv);
    for (int i = 0; i < nv; ++i) {
        float o[4];
        m4v(s->object_to_render, s->positions[3 * i], s->positions[3 * i + 1], s->positions[3 * i + 2], 1.f, o);
        w.wv[i] = {o[0], o[1], o[2]};
    }
    w.tri3.resize(3 * (size_t)nt);
    for (int t = 0; t < nt; ++t)
        for (int k = 0; k < 3; ++k) w.tri3[3 * (size_t)t + k] = w.wv[s->indices[3 * t + k]];
    w.back.assign(nt, 0);
    w.degen.assign(nt, 0);
    const bool cull = s->cull_backfaces != 0;
    F3 look = f3norm({s->cull_look[0], s->cull_look[1], s->cull_look[2]});
    for (int t = 0; t < nt; ++t) {
        const F3* p = &w.tri3[3 * (size_t)t];
        F3 cr = f3cross(f3sub(p[2], p[0]), f3sub(p[1], p[0]));
        w.degen[t] = f3dot(cr, cr) == 0;
        if (cull) {
            F3 n[3];
            for (int k = 0; k < 3; ++k) {
                uint32_t v = s->indices[3 * t + k];
                n[k] = {s->normals[3 * v], s->normals[3 * v + 1], s->normals[3 * v + 2]};
            }
            F3 sum = f3add(f3add(n[0], n[1]), n[2]);
            F3 N = f3norm({sum.x / 3.0f, sum.y / 3.0f, sum.z / 3.0f});
            N = f3norm(m3v(s->normal_to_render, N));
            w.back[t] = f3dot(look, N) > 0;
        }
    }
}
// The fast traversal's BVH over tile set `set` (non-degenerate triangles; set 1 without the back-facing ones) and
// the canonical rule's constants, from M = max |world vertex coordinate|:
//   wabs = M 2^-20 (the window W(t) = t 2^-16 + wabs; the oracle's Octree::SetWindow computes the same value);
//   pad = M 2^-18: every child box is padded by it before quantisation.  The slab test's rounding (box_entry in
//     rt_kernels.hip: base = fma(origin, inv, -o inv), t = fma(q, inv 2^e, base)) moves a plane by at most a few
//     ulp of max(|o|, M) along its axis, i.e. < 2^-21 max(|o|, M), well inside the pad while |o| <= 8 M;
//   oguard = 8 M: rays whose origin lies farther out in some coordinate are declared ambiguous (exact BFS).
static void scene_bvh(const SceneWorld& w, int set, float node_cost, int max_leaf, BvhData& out, float& wabs,
                      float& oguard) {
    float mc = 0.f;
    for (const F3& p : w.wv) mc = std::max(mc, std::max(std::fabs(p.x), std::max(std::fabs(p.y), std::fabs(p.z))));
    wabs = mc * 0x1p-20f;
    oguard = mc * 8.f;
    const float pad = mc * 0x1p-18f;
    const int nt = (int)w.degen.size();
    std::vector<float> t9;
    std::vector<int> ids;
    for (int t = 0; t < nt; ++t) {
        if (w.degen[t] || (set == 1 && w.back[t])) continue;
        for (int k = 0; k < 3; ++k) {
            const F3& p = w.tri3[3 * (size_t)t + k];
            t9.push_back(p.x); t9.push_back(p.y); t9.push_back(p.z);
        }
        ids.push_back(t);
    }
    build_bvh8(t9.data(), ids.data(), (int)ids.size(), pad, node_cost, out, max_leaf);
}

static int scene_upload_one(rt_ctx* c, const rt_scene_desc* s) {
    if (!c || !s) return RT_E_ARG;
    if (s->n_triangles <= 0 || s->n_vertices <= 0 || !s->positions || !s->indices)
        return fail(c, RT_E_ARG, "scene needs positions and indices");
    if (s->cull_backfaces && !s->normals) return fail(c, RT_E_ARG, "back-face culling needs vertex normals");
    for (int t = 0; t < 3 * s->n_triangles; ++t)
        if (s->indices[t] >= (uint32_t)s->n_vertices) return fail(c, RT_E_ARG, "triangle index out of range");
    if (s->tri_material)
        for (int t = 0; t < s->n_triangles; ++t)
            if (s->tri_material[t] < 0 || s->tri_material[t] >= std::max(1, s->n_materials))
                return fail(c, RT_E_ARG, "material id out of range");
    auto mat_ok = [&](int m) { return m >= 0 && m < std::max(1, s->n_materials); };
    for (int i = 0; i < s->n_materials; ++i) {
        const rt_material& m = s->materials[i];
        if (m.type < RT_MAT_DIFFUSE || m.type > RT_MAT_DIELECTRIC) return fail(c, RT_E_ARG, "unknown material type");
        if (m.type == RT_MAT_DIELECTRIC && m.eta < 0) return fail(c, RT_E_ARG, "dielectric eta must be >= 0");
    }
    if (s->n_shapes < 0 || (s->n_shapes > 0 && !s->shapes)) return fail(c, RT_E_ARG, "shapes");
    for (int i = 0; i < s->n_shapes; ++i) {
        const rt_shape& h = s->shapes[i];
        if (!mat_ok(h.material)) return fail(c, RT_E_ARG, "shape material out of range");
        if (h.type == RT_SHAPE_SPHERE) {
            if (!(h.radius > 0) || h.zmin > -h.radius || h.zmax < h.radius || h.phimax < 360.f)
                return fail(c, RT_E_ARG, "only full spheres are supported (zmin <= -r, zmax >= r, phimax >= 360)");
        } else if (h.type == RT_SHAPE_DISK) {
            if (h.phimax < 360.f || !(h.outer_radius > 0) || h.inner_radius < 0)
                return fail(c, RT_E_ARG, "only full disks are supported (phimax >= 360)");
        } else if (h.type != RT_SHAPE_TRIANGLE) {
            return fail(c, RT_E_ARG, "unknown shape type");
        }
    }
    if (s->n_lights < 0 || s->n_lights > kMaxLights || (s->n_lights > 0 && !s->lights))
        return fail(c, RT_E_ARG, "lights: at most " + std::to_string(kMaxLights));
    for (int i = 0; i < s->n_lights; ++i) {
        const rt_light& L = s->lights[i];
        if (L.type == RT_LIGHT_QUAD) {
            if (!mat_ok(L.material) || !(s->materials && s->materials[L.material].emission_scale > 0))
                return fail(c, RT_E_ARG, "quad light needs an emissive material");
        } else if (L.type == RT_LIGHT_DISK) {
            if (L.shape < 0 || L.shape >= s->n_shapes || s->shapes[L.shape].type != RT_SHAPE_DISK ||
                s->shapes[L.shape].inner_radius != 0 || !(s->materials[s->shapes[L.shape].material].emission_scale > 0))
                return fail(c, RT_E_ARG, "disk light needs an emissive full DISK shape with inner radius 0");
        } else if (L.type == RT_LIGHT_DISTANT) {
            if (L.dir[0] == 0 && L.dir[1] == 0 && L.dir[2] == 0) return fail(c, RT_E_ARG, "distant light direction");
        } else if (L.type != RT_LIGHT_POINT) {
            return fail(c, RT_E_ARG, "unknown light type");
        }
    }
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    free_scene(c);
    const int nt = s->n_triangles, nv = s->n_vertices;
    SceneWorld sw;
    scene_world(s, sw);
    const std::vector<F3>& tri3 = sw.tri3;
    const std::vector<uint8_t>&back = sw.back, &degen = sw.degen;
    c->cull = s->cull_backfaces != 0;
    // root bounds: TriModel::Bounds (Shapes.h:1390-1397): object-space min/max (max starts at FLT_MIN, :1292)
    // then Bounds3::Transform (Shapes.h:60-98, same FLT_MIN quirk)
    const float FMAX = std::numeric_limits<float>::max(), FMIN = std::numeric_limits<float>::min();
    F3 omn = {FMAX, FMAX, FMAX}, omx = {FMIN, FMIN, FMIN};
    for (int i = 0; i < nv; ++i) {
        const float* p = s->positions + 3 * i;
        omn = {std::min(omn.x, p[0]), std::min(omn.y, p[1]), std::min(omn.z, p[2])};
        omx = {std::max(omx.x, p[0]), std::max(omx.y, p[1]), std::max(omx.z, p[2])};
    }
    const F3 corners[8] = {{omn.x, omn.y, omn.z}, {omn.x, omx.y, omn.z}, {omn.x, omx.y, omx.z}, {omn.x, omn.y, omx.z},
                           {omx.x, omx.y, omx.z}, {omx.x, omn.y, omx.z}, {omx.x, omn.y, omn.z}, {omx.x, omx.y, omn.z}};
    F3 rmn = {FMAX, FMAX, FMAX}, rmx = {FMIN, FMIN, FMIN};
    for (const F3& q : corners) {
        float o[4];
        m4v(s->object_to_render, q.x, q.y, q.z, 1.f, o);
        rmn = {std::min(rmn.x, o[0]), std::min(rmn.y, o[1]), std::min(rmn.z, o[2])};
        rmx = {std::max(rmx.x, o[0]), std::max(rmx.y, o[1]), std::max(rmx.z, o[2])};
    }
    {  // ray coherence sort: origins quantised to 9 bits per axis over the root box
        F3 e = f3sub(rmx, rmn);
        auto sc = [](float x) { return x > 0 ? 512.0f / x : 0.0f; };
        c->sort_lo = make_float4(rmn.x, rmn.y, rmn.z, 0.f);
        c->sort_scale = make_float4(sc(e.x), sc(e.y), sc(e.z), 0.f);
    }
    // octree build (all triangles, culled and degenerate included — the reference inserts every triangle)
    OctBuild ob;
    ob.tri3 = &tri3;
    ob.capacity = s->octree_capacity > 0 ? s->octree_capacity : 40;
    OctBuild::Node root;
    root.mn = rmn;
    root.mx = rmx;
    ob.nodes.push_back(root);
    if (c->octree_build == RT_OCTREE_BUILD_HOST) {
        for (int t = 0; t < nt; ++t) ob.add(t);
    } else {
        std::string err;
        int brc = octree_build_device(c->stream, ob, nt, err);
        if (brc) return fail(c, brc, err);
    }
    const int nn = (int)ob.nodes.size();
    // flatten: node SoA + two tile sets
    std::vector<float4> nA(nn), nB(nn);
    std::vector<int2> lr0(nn), lr1(nn);
    std::vector<float4> tiles0, tiles1;
    c->h_bounds.assign(6 * (size_t)nn, 0.f);
    c->h_child.assign(nn, -1);
    c->h_leaf_first.assign(nn, 0);
    c->h_leaf_count.assign(nn, 0);
    c->h_refs.clear();
    auto push_tile = [&](std::vector<float4>& v, int t) {
        const F3* p = &tri3[3 * (size_t)t];
        int bits = t;
        float fid;
        std::memcpy(&fid, &bits, 4);
        v.push_back(make_float4(p[0].x, p[0].y, p[0].z, p[1].x));
        v.push_back(make_float4(p[1].y, p[1].z, p[2].x, p[2].y));
        v.push_back(make_float4(p[2].z, fid, 0.f, 0.f));
    };
    for (int i = 0; i < nn; ++i) {
        const auto& N = ob.nodes[i];
        int child = N.first_child;
        float fc;
        std::memcpy(&fc, &child, 4);
        nA[i] = make_float4(N.mn.x, N.mn.y, N.mn.z, fc);
        nB[i] = make_float4(N.mx.x, N.mx.y, N.mx.z, 0.f);
        float* b = &c->h_bounds[6 * (size_t)i];
        b[0] = N.mn.x; b[1] = N.mn.y; b[2] = N.mn.z; b[3] = N.mx.x; b[4] = N.mx.y; b[5] = N.mx.z;
        c->h_child[i] = child;
        c->h_leaf_first[i] = (int)c->h_refs.size();
        c->h_leaf_count[i] = (int)N.tris.size();
        lr0[i] = make_int2((int)tiles0.size() / 3, 0);
        lr1[i] = make_int2((int)tiles1.size() / 3, 0);
        for (int t : N.tris) {
            c->h_refs.push_back(t);
            if (degen[t]) continue;
            push_tile(tiles0, t);
            lr0[i].y++;
            if (!back[t]) { push_tile(tiles1, t); lr1[i].y++; }
        }
    }
    // BFS group-queue bound: max over depth d of (#internal nodes at d-1 + #internal nodes at d)
    std::vector<int> depth(nn, 0), internal_at;
    int maxd = 0;
    for (int i = 0; i < nn; ++i) {
        if (ob.nodes[i].first_child >= 0)
            for (int k = 0; k < 8; ++k) depth[ob.nodes[i].first_child + k] = depth[i] + 1;
        maxd = std::max(maxd, depth[i]);
    }
    internal_at.assign(maxd + 2, 0);
    for (int i = 0; i < nn; ++i)
        if (ob.nodes[i].first_child >= 0) internal_at[depth[i]]++;
    // Exact worst case of the kernel's group FIFO: replay the BFS with every box test passing (any real ray
    // pushes a subset of these groups, in the same order, so its queue is never longer at the same point).
    int bound = 0;
    {
        std::vector<int> fifo;
        fifo.reserve(nn);
        size_t head = 0;
        int cur = 0, left = 1;
        while (true) {
            int fc = ob.nodes[cur].first_child;
            if (fc >= 0) {
                fifo.push_back(fc);
                bound = std::max(bound, (int)(fifo.size() - head));
            }
            if (--left > 0) { ++cur; continue; }
            if (head == fifo.size()) break;
            cur = fifo[head++];
            left = 8;
        }
    }
    int qcap = 1;
    if (ob.nodes[0].first_child >= 0) {
        const int caps[] = {16};  // register FIFO; larger bounds use the LDS + HBM-spill FIFO (qcap 0)
        qcap = 0;
        for (int cp : caps)
            if (cp >= bound) { qcap = cp; break; }
        if (!qcap && bound > kRingMax)
            return fail(c, RT_E_LIMIT, "octree BFS frontier bound " + std::to_string(bound) + " exceeds " +
                                           std::to_string(kRingMax) + " groups");
        // the LDS FIFO stores 16-bit group ids: children are created 8 at a time after the root (node 1 + 8 g)
        for (int i = 0; i < nn && !qcap; ++i) {
            int fc = ob.nodes[i].first_child;
            if (fc >= 0 && ((fc - 1) % 8 != 0 || (fc - 1) / 8 > 65535))
                return fail(c, RT_E_LIMIT, "octree too large for 16-bit BFS group ids");
        }
    }
    // multi-level octrees: the fast traversal's BVH per tile set (non-degenerate triangles; set 1 without the
    // back-facing ones) and the canonical-rule window (rt_bvh.cpp)
    // [kBvhAny]: the any-hit BVH of the shadow rays (set 0), built with its own SAH cost and leaf size
    BvhData bvh[3];
    float wabs = 0.f, oguard = 0.f;
    if (qcap != 1) {
        // a BVH leaf word holds its first tile in 27 bits (rt_kernels.hip decode_leaf): one tile per triangle
        if (sw.tri3.size() / 3 >= ((size_t)1 << 27))
            return fail(c, RT_E_LIMIT, "more than 2^27 triangles: the BVH leaf words hold 27-bit tile offsets");
        for (int st = 0; st < (c->cull ? 2 : 1); ++st)
            scene_bvh(sw, st, c->bvh_node_cost, c->bvh_max_leaf, bvh[st], wabs, oguard);
        if (c->bvh_any_cost > 0) scene_bvh(sw, 0, c->bvh_any_cost, c->bvh_any_leaf, bvh[kBvhAny], wabs, oguard);
    } else {
        // single leaf: the same window for the closest-hit pass 2's nearest-first order (rt_kernels.hip traverse)
        float mc = 0.f;
        for (const F3& p : sw.wv) mc = std::max(mc, std::max(std::fabs(p.x), std::max(std::fabs(p.y), std::fabs(p.z))));
        wabs = mc * 0x1p-20f;
    }
    c->info.n_nodes = nn;
    c->info.n_leaf_refs = (int)c->h_refs.size();
    c->info.max_queue_groups = bound;
    c->info.depth = maxd;
    c->n_tris = nt;
    // per-triangle shading data
    std::vector<float4> tw(3 * (size_t)nt), tn(3 * (size_t)nt);
    for (int t = 0; t < nt; ++t)
        for (int k = 0; k < 3; ++k) {
            const F3& p = tri3[3 * (size_t)t + k];
            tw[3 * (size_t)t + k] = make_float4(p.x, p.y, p.z, 0.f);
            uint32_t v = s->indices[3 * t + k];
            tn[3 * (size_t)t + k] = s->normals ? make_float4(s->normals[3 * v], s->normals[3 * v + 1], s->normals[3 * v + 2], 0.f)
                                               : make_float4(0.f, 0.f, 1.f, 0.f);
        }
    std::vector<int> tm(nt, 0);
    if (s->tri_material) tm.assign(s->tri_material, s->tri_material + nt);
    std::vector<DevMaterial> mats;
    for (int i = 0; i < s->n_materials; ++i) {
        const rt_material& m = s->materials[i];
        const int cls = m.emission_scale > 0 || m.type == RT_MAT_DIFFUSE ? 0 : 1;  // material bin (kMatClasses)
        mats.push_back(DevMaterial{m.sigmoid[0], m.sigmoid[1], m.sigmoid[2], m.emission_scale, m.type, m.eta, -1, cls});
    }
    if (mats.empty()) mats.push_back(DevMaterial{0.f, 0.f, 0.f, 0.f, RT_MAT_DIFFUSE, 0.f, -1, 0});
    std::vector<DevShape> shapes(s->n_shapes);
    for (int i = 0; i < s->n_shapes; ++i) {
        const rt_shape& h = s->shapes[i];
        DevShape& d = shapes[i];
        d = DevShape{};
        d.type = h.type; d.material = h.material; d.light = -1;
        d.r = h.radius;
        d.zmin = std::min(std::max(h.zmin, -h.radius), h.radius);  // glm::clamp(_zmin, -r, r) (Shapes.h:222-223)
        d.zmax = std::min(std::max(h.zmax, -h.radius), h.radius);
        d.h = h.height; d.ri = h.inner_radius; d.ro = h.outer_radius;
        std::memcpy(d.o2r, h.object_to_render, 64); std::memcpy(d.r2o, h.render_to_object, 64);
        std::memcpy(d.n2r, h.normal_to_render, 36);
        std::memcpy(d.p1, h.p, 12); std::memcpy(d.p2, h.p + 3, 12); std::memcpy(d.p3, h.p + 6, 12);
        shape_bound(d);
    }
    std::vector<DevLight> lights(s->n_lights);
    bool full = s->n_shapes > 0 || s->n_lights != 1;
    for (const DevMaterial& m : mats) full = full || m.type != RT_MAT_DIFFUSE;
    for (int i = 0; i < s->n_lights; ++i) {
        const rt_light& q = s->lights[i];
        DevLight& L = lights[i];
        L = DevLight{};
        L.type = q.type; L.shape = q.shape; L.material = q.material; L.scale = q.scale;
        for (int k = 0; k < 3; ++k) { L.p[k] = q.p[k]; L.e1[k] = q.e1[k]; L.e2[k] = q.e2[k]; L.n[k] = q.n[k]; }
        if (q.type == RT_LIGHT_QUAD) {
            F3 cr = f3cross({q.e1[0], q.e1[1], q.e1[2]}, {q.e2[0], q.e2[1], q.e2[2]});
            L.area = std::sqrt(f3dot(cr, cr));
            if (mats[q.material].light < 0) mats[q.material].light = i;
        } else if (q.type == RT_LIGHT_DISK) {
            const DevShape& ds = shapes[q.shape];
            const float phimax = 360.0f * 0.01745329251994329576923690768489f;  // glm::radians(360.f)
            L.area = phimax * .5f * (ds.ro * ds.ro - ds.ri * ds.ri);           // Disk::Area (Shapes.h:641-644)
            F3 n = f3norm(m3v(ds.n2r, F3{0.f, 0.f, 1.f}));
            L.n[0] = n.x; L.n[1] = n.y; L.n[2] = n.z;
            L.material = ds.material; L.ro = ds.ro; L.h = ds.h;
            std::memcpy(L.o2r, ds.o2r, 64);
            shapes[q.shape].light = i;
        } else if (q.type == RT_LIGHT_DISTANT) {
            F3 d = f3norm(F3{q.dir[0], q.dir[1], q.dir[2]});
            L.dir[0] = d.x; L.dir[1] = d.y; L.dir[2] = d.z;
        }
        if (q.type != RT_LIGHT_QUAD) full = true;
    }
    // upload
    auto up = [&](const void* src, size_t bytes, void** dst) -> int {
        void* p = nullptr;
        HIPCHK(c, hipMalloc(&p, std::max<size_t>(bytes, 16)));
        c->scene_allocs.push_back(p);
        if (bytes) HIPCHK(c, hipMemcpy(p, src, bytes, hipMemcpyHostToDevice));
        *dst = p;
        return RT_OK;
    };
    void *pA, *pB, *pl0, *pl1, *pt0, *pt1 = nullptr, *ptw, *ptn, *ptm, *pm, *psh, *plt;
    int rc;
    if ((rc = up(nA.data(), nA.size() * 16, &pA)) || (rc = up(nB.data(), nB.size() * 16, &pB)) ||
        (rc = up(lr0.data(), lr0.size() * 8, &pl0)) || (rc = up(lr1.data(), lr1.size() * 8, &pl1)) ||
        (rc = up(tiles0.data(), tiles0.size() * 16, &pt0)) || (rc = up(tiles1.data(), tiles1.size() * 16, &pt1)) ||
        (rc = up(tw.data(), tw.size() * 16, &ptw)) || (rc = up(tn.data(), tn.size() * 16, &ptn)) ||
        (rc = up(tm.data(), tm.size() * 4, &ptm)) || (rc = up(mats.data(), mats.size() * sizeof(DevMaterial), &pm)) ||
        (rc = up(shapes.data(), shapes.size() * sizeof(DevShape), &psh)) ||
        (rc = up(lights.data(), lights.size() * sizeof(DevLight), &plt)))
        return rc;
    // single-leaf octree: conservative boxes of runs of kClusterTris leaf tiles (pass-1 culling in the kernel); a
    // box miss means none of its triangles can pass the watertight test's tMax-independent checks, so the
    // inflation only has to cover those checks' rounding.  In the sheared frame every vertex coordinate carries
    // at most ~4 ulp(M) of error, M = the largest |vertex - origin|; with origins inside 8 extents of the scene
    // centre (cl_guard; farther rays never skip) M <= 9.8 ext, i.e. <= 2.4e-6 ext, and the pad is 1e-5 ext +
    // 1e-3 — small enough that a wave of rays leaving one wall (origin offset 1e-4 (1 + max|p|)) skips it.
    std::vector<float4> clus[2];
    if (qcap == 1) {
        const std::vector<float4>* tl[2] = {&tiles0, &tiles1};
        const auto& R = ob.nodes[0];
        float ext = std::max(std::max(R.mx.x - R.mn.x, R.mx.y - R.mn.y), R.mx.z - R.mn.z);
        float pad = kClusterPadRel * ext + 1e-3f;
        c->dsc.cl_guard = make_float4(.5f * (R.mn.x + R.mx.x), .5f * (R.mn.y + R.mx.y), .5f * (R.mn.z + R.mx.z),
                                      64.f * ext * ext);
        for (int st = 0; st < 2; ++st) {
            int nt_leaf = (int)tl[st]->size() / 3;
            for (int k0 = 0; k0 < nt_leaf; k0 += kClusterTris) {
                float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
                for (int k = k0; k < std::min(nt_leaf, k0 + kClusterTris); ++k) {
                    const float4* q = tl[st]->data() + 3 * k;
                    float v[9] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w, q[2].x};
                    for (int j = 0; j < 3; ++j)
                        for (int a = 0; a < 3; ++a) { mn[a] = std::min(mn[a], v[3 * j + a]); mx[a] = std::max(mx[a], v[3 * j + a]); }
                }
                clus[st].push_back(make_float4(mn[0] - pad, mn[1] - pad, mn[2] - pad, 0.f));
                clus[st].push_back(make_float4(mx[0] + pad, mx[1] + pad, mx[2] + pad, 0.f));
            }
            c->dsc.n_clusters[st] = (int)clus[st].size() / 2;
            // fan pairs: tile k+1 = (a, c, d) after tile k = (a, b, c), bit for bit (_quad / OBJ fan triangulation)
            unsigned long long fp = 0;
            for (int k = 0; k + 1 < std::min(nt_leaf, 64); k += 2) {
                const float4* q = tl[st]->data() + 3 * k;
                float v[9] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w, q[2].x};
                float w[9] = {q[3].x, q[3].y, q[3].z, q[3].w, q[4].x, q[4].y, q[4].z, q[4].w, q[5].x};
                if (!std::memcmp(w, v, 12) && !std::memcmp(w + 3, v + 6, 12)) fp |= 1ull << k;
            }
            c->dsc.fan_pairs[st] = fp;
        }
    }
    void *pc0 = nullptr, *pc1 = nullptr;
    if ((rc = up(clus[0].data(), clus[0].size() * 16, &pc0)) || (rc = up(clus[1].data(), clus[1].size() * 16, &pc1)))
        return rc;
    void* pbv[3] = {nullptr, nullptr, nullptr};
    void* pbt[3] = {nullptr, nullptr, nullptr};
    void* pbi[3] = {nullptr, nullptr, nullptr};
    const int bvh_nodes0 = (int)(bvh[0].nodes.size() / kBvhNodeF4);
    for (int st = 0; st < 3; ++st) {
        // a BVH not built here (no culled set; the any-hit walks on the closest-hit BVH of set 0) uses set 0's arrays
        const int src = bvh[st].nodes.empty() ? 0 : st;
        c->bvh_count[st][0] = (int)(bvh[src].nodes.size() / kBvhNodeF4);
        c->bvh_count[st][1] = (int)bvh[src].tid.size();
    }
    for (int st = 0; st < 3; ++st) {
        if (bvh[st].nodes.empty()) continue;
        // the kernels stage nodes [0, kBvhTopNodes) in LDS unconditionally: pad with empty nodes
        if (bvh[st].nodes.size() < kBvhNodeF4 * (size_t)kBvhTopNodes)
            bvh[st].nodes.resize(kBvhNodeF4 * (size_t)kBvhTopNodes, make_float4(0.f, 0.f, 0.f, 0.f));
        bvh[st].tiles.resize(bvh[st].tiles.size() + 4, 0.f);  // (an empty BVH still gets a buffer)
        bvh[st].tid.push_back(-1);
        if ((rc = up(bvh[st].nodes.data(), bvh[st].nodes.size() * 16, &pbv[st])) ||
            (rc = up(bvh[st].tiles.data(), bvh[st].tiles.size() * 4, &pbt[st])) ||
            (rc = up(bvh[st].tid.data(), bvh[st].tid.size() * 4, &pbi[st])))
            return rc;
    }
    DevScene& d = c->dsc;
    for (int st = 0; st < 3; ++st) {
        d.bvh[st] = (const float4*)(pbv[st] ? pbv[st] : pbv[0]);
        d.btiles[st] = (const float*)(pbt[st] ? pbt[st] : pbt[0]);
        d.btid[st] = (const int*)(pbi[st] ? pbi[st] : pbi[0]);
    }
    d.wabs = wabs;
    d.oguard = oguard;
    d.amb_force = c->force_amb >= 0;
    d.amb_mask = c->force_amb > 0 ? (1u << c->force_amb) - 1u : 0u;
    c->info.bvh_nodes = bvh_nodes0;
    c->info.bvh_depth = bvh[0].depth;
    d.clusters[0] = (const float4*)pc0; d.clusters[1] = (const float4*)pc1;
    if (qcap != 1) d.n_clusters[0] = d.n_clusters[1] = 0;
    d.nodeA = (const float4*)pA; d.nodeB = (const float4*)pB;
    d.leafRange[0] = (const int2*)pl0; d.leafRange[1] = (const int2*)pl1;
    d.tiles[0] = (const float4*)pt0; d.tiles[1] = (const float4*)pt1;
    d.triWorld = (const float4*)ptw; d.triNormal = (const float4*)ptn;
    d.triMaterial = (const int*)ptm; d.materials = (const DevMaterial*)pm;
    d.shapes = (const DevShape*)psh; d.lights = (const DevLight*)plt;
    d.n_nodes = nn;
    d.n_tris = nt;
    d.n_shapes = s->n_shapes;
    d.n_materials = (int)mats.size();
    c->scene_full = full;
    d.qcap = qcap;
    {  // the cooperative BFS's FIFO holds 16-bit group ids (first child = 1 + 8 g) and kCoopFifo of them
        bool ids16 = true;
        for (int i = 0; i < nn && ids16; ++i) {
            const int fc = ob.nodes[i].first_child;
            if (fc >= 0 && ((fc - 1) % 8 != 0 || (fc - 1) / 8 > 65535)) ids16 = false;
        }
        d.coop_ok = c->coop && qcap != 1 && bound <= kCoopFifo && ids16 ? 1 : 0;
    }
    d.depth = nn < (1 << 24) ? maxd : 1 << 30;  // DFS stack entries hold 24-bit group ids
    if (qcap == 0) {  // each lane allocates its ring of ring_threads x rs ints (ensure_ring)
        int rs = 1;
        while (rs < bound) rs <<= 1;
        d.ring_threads = c->grid * kBlockThreads;
        d.ring_mask = rs - 1;
    }
    d.n_lights = s->n_lights;
    if (s->n_lights >= 1) d.light0 = lights[0];
    // the emissive surfaces, for the last depth's emitter filter (EmitIO): non-degenerate triangles and shapes whose
    // material emits; more than kMaxEmitTris emissive triangles turn the filter off
    std::vector<int> etris, eshapes;
    for (int t = 0; t < nt; ++t)
        if (!degen[t] && mats[tm[t]].emit > 0) etris.push_back(t);
    for (int i = 0; i < s->n_shapes; ++i)
        if (mats[shapes[i].material].emit > 0) eshapes.push_back(i);
    void *pet = nullptr, *pes = nullptr;
    if ((rc = up(etris.data(), etris.size() * 4, &pet)) || (rc = up(eshapes.data(), eshapes.size() * 4, &pes)))
        return rc;
    d.emit_tris = (const int*)pet;
    d.n_emit_tris = (int)etris.size() <= kMaxEmitTris ? (int)etris.size() : -1;
    d.emit_shapes = (const int*)pes;
    d.n_emit_shapes = (int)eshapes.size();
    c->have_scene = true;
    return RT_OK;
}

static int camera_set_one(rt_ctx* c, const rt_camera_desc* d) {
    if (!c || !d) return RT_E_ARG;
    if (d->type < RT_CAMERA_PERSPECTIVE || d->type > RT_CAMERA_THINLENS) return fail(c, RT_E_ARG, "unknown camera type");
    c->cam = *d;
    c->have_cam = true;
    return RT_OK;
}

static int sampler_set_one(rt_ctx* c, const rt_sampler_desc* d) {
    if (!c || !d) return RT_E_ARG;
    if (d->kind < RT_SAMPLER_INDEPENDENT || d->kind > RT_SAMPLER_SOBOL) return fail(c, RT_E_ARG, "unknown sampler");
    if (d->kind == RT_SAMPLER_SOBOL && (d->randomize < RT_SOBOL_NONE || d->randomize > RT_SOBOL_OWEN))
        return fail(c, RT_E_ARG, "unknown Sobol randomization");
    if (d->x_samples <= 0 || (d->kind == RT_SAMPLER_STRATIFIED && d->y_samples <= 0))
        return fail(c, RT_E_ARG, "samples per pixel must be positive");
    c->smp = *d;
    c->have_smp = true;
    return RT_OK;
}

static int film_set_one(rt_ctx* c, const rt_film_desc* d) {
    if (!c || !d) return RT_E_ARG;
    if (d->res_x <= 0 || d->res_y <= 0 || d->filter < RT_FILTER_BOX || d->filter > RT_FILTER_LANCZOS)
        return fail(c, RT_E_ARG, "invalid film");
    if ((size_t)d->res_x * d->res_y > ((size_t)1 << 27)) return fail(c, RT_E_LIMIT, "film too large");
    if (d->sensor < 0 || d->sensor >= RT_SENSOR_COUNT || d->sensor_illum < 0 || d->sensor_illum >= RT_ILLUM_COUNT)
        return fail(c, RT_E_ARG, "unknown sensor or sensor illuminant");
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);  // queued passes may still read the old tables
    int y_int = 0;  // committed with the film descriptor below, only once the sensor is set up
    {  // RayTracerTestApp.h:289-291 divides in float; the kernels may divide integers where that is identical
        const int w = d->res_x, n = d->res_x * d->res_y;
        int ok = 1;
        for (int p = 0; p < n && ok; ++p) ok = (int)std::floor((float)p / (float)w) == p / w;
        y_int = ok;
    }
    int rc = setup_sensor(c, *d);
    if (rc) return rc;
    if (c->d_cdf) { hipFree(c->d_cdf); c->d_cdf = nullptr; c->cdf_n = 0; }
    if (d->filter == RT_FILTER_GAUSSIAN || d->filter == RT_FILTER_LANCZOS) {
        std::vector<float> tx, ty;
        int n = build_filter_tables(*d, tx, ty);
        if (hipMalloc(&c->d_cdf, sizeof(float) * 2 * (n + 1)) != hipSuccess) return fail(c, RT_E_OOM, "filter tables");
        hipMemcpy(c->d_cdf, tx.data(), sizeof(float) * (n + 1), hipMemcpyHostToDevice);
        hipMemcpy(c->d_cdf + (n + 1), ty.data(), sizeof(float) * (n + 1), hipMemcpyHostToDevice);
        c->cdf_n = n;
    }
    c->film = *d;
    c->film_y_int = y_int;
    c->have_film = true;
    c->work_dirty = true;
    return RT_OK;
}

static_assert(rtdata::n_cameras + 1 == RT_SENSOR_COUNT, "camera table and RT_SENSOR_COUNT disagree");

const char* rt_sensor_name(int sensor) {
    if (sensor == RT_SENSOR_XYZ) return "xyz";
    if (sensor < 1 || sensor >= RT_SENSOR_COUNT) return nullptr;
    return rtdata::camera_names[sensor - 1];
}

static int impl_rt_film_matrices(rt_ctx* c, float* xyz_from_sensor9, float* rgb_from_xyz9) {
    if (!c || !xyz_from_sensor9 || !rgb_from_xyz9) return RT_E_ARG;
    std::memcpy(xyz_from_sensor9, c->resolveA, 36);
    std::memcpy(rgb_from_xyz9, c->resolveB, 36);
    return RT_OK;
}

static int integrator_set_one(rt_ctx* c, const rt_integrator_desc* d) {
    if (!c || !d) return RT_E_ARG;
    if (d->kind != RT_INTEGRATOR_REFERENCE && d->kind != RT_INTEGRATOR_PATH && d->kind != RT_INTEGRATOR_PATH_MIS)
        return fail(c, RT_E_ARG, "unknown integrator");
    if (d->max_depth < 0 || d->max_depth > 64) return fail(c, RT_E_ARG, "max_depth out of range");
    if (d->kind == RT_INTEGRATOR_REFERENCE &&
        !(d->albedo_rgb[0] == d->albedo_rgb[1] && d->albedo_rgb[1] == d->albedo_rgb[2] && d->albedo_rgb[0] > 0 &&
          d->albedo_rgb[0] < 1))
        return fail(c, RT_E_ARG, "reference Li albedo must be a grey in (0,1): the RGB->spectrum table is absent "
                                 "(color.cpp:114), only the uniform branch color.cpp:35-37 exists");
    c->integ = *d;
    c->have_integ = true;
    return RT_OK;
}

static int set_shard_one(rt_ctx* c, int tile_size, int n_shards, int shard_id) {
    if (!c || tile_size <= 0 || tile_size % 8 || n_shards <= 0 || shard_id < 0 || shard_id >= n_shards)
        return c ? fail(c, RT_E_ARG, "invalid shard (tile_size must be a positive multiple of 8)") : RT_E_ARG;
    c->tile = tile_size;
    c->n_shards = n_shards;
    c->shard_id = shard_id;
    c->work_dirty = true;
    return RT_OK;
}

static int impl_rt_render_pass_device(rt_ctx* c, int ib, int ie, void* d_film, void* stream) {
    if (!c || !d_film) return RT_E_ARG;
    hipSetDevice(c->device);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return render_multi(c, ib, ie, (float4*)d_film, st);
}

static int impl_rt_render_pass(rt_ctx* c, int ib, int ie, rt_pixel* film) {
    if (!c || !film) return RT_E_ARG;
    int rc = check_ready(c);
    if (rc) return rc;
    hipSetDevice(c->device);
    size_t n = (size_t)c->film.res_x * c->film.res_y;
    if (c->film_cap < n) {
        if (c->d_film) hipFree(c->d_film);
        c->d_film = nullptr;
        HIPCHK(c, dalloc(&c->d_film, n));
        c->film_cap = n;
    }
    HIPCHK(c, hipMemcpyAsync(c->d_film, film, n * 16, hipMemcpyHostToDevice, c->stream));
    if ((rc = render_multi(c, ib, ie, c->d_film, c->stream))) return rc;
    HIPCHK(c, hipMemcpyAsync(film, c->d_film, n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

namespace {
int film_resolve(rt_ctx* c, const rt_pixel* film, uint8_t* out, int srgb) {
    if (!c || !film || !out) return RT_E_ARG;
    if (!c->have_film) return fail(c, RT_E_STATE, "film not set");
    hipSetDevice(c->device);
    size_t n = (size_t)c->film.res_x * c->film.res_y;
    float4* df = nullptr;
    unsigned char* dout = nullptr;
    HIPCHK(c, dalloc(&df, n));
    if (dalloc(&dout, 3 * n) != hipSuccess) { hipFree(df); return fail(c, RT_E_OOM, "resolve buffer"); }
    int rc = RT_OK;
    if (hipMemcpy(df, film, n * 16, hipMemcpyHostToDevice) != hipSuccess ||
        launch_resolve(c->stream, (int)n, df, c->d_resolve, c->d_resolve + 9, dout, srgb) != hipSuccess ||
        hipMemcpyAsync(out, dout, 3 * n, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        rc = fail(c, RT_E_HIP, "resolve failed");
    hipFree(df);
    hipFree(dout);
    return rc;
}
}  // namespace

static int impl_rt_film_resolve(rt_ctx* c, const rt_pixel* film, uint8_t* out) { return film_resolve(c, film, out, 0); }
static int impl_rt_film_resolve_srgb(rt_ctx* c, const rt_pixel* film, uint8_t* out) { return film_resolve(c, film, out, 1); }

static int get_stats_one(rt_ctx* c, rt_stats* out) {
    if (!c || !out) return RT_E_ARG;
    hipSetDevice(c->device);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipDeviceSynchronize());
    harvest(c);
    std::vector<unsigned long long> raw(kCtrWords);
    HIPCHK(c, hipMemcpy(raw.data(), c->d_ctr, kCtrWords * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    unsigned long long h[C_NCOUNTERS] = {};
    for (int k = 0; k < C_NCOUNTERS; ++k)
        for (int u = 0; u < kCtrSubs; ++u) h[k] += raw[ctr_word(k, u)];
    rt_stats s = c->stats;
    s.nodes_tested = (int64_t)h[C_NODES];
    s.tris_tested = (int64_t)h[C_TRIS];
    s.hits = (int64_t)h[C_HITS];
    s.rays = (int64_t)h[C_RAYS];
    s.shadow_rays = (int64_t)h[C_SHADOW];
    s.shadow_nodes_tested = (int64_t)h[C_SNODES];
    s.shadow_tris_tested = (int64_t)h[C_STRIS];
    s.samples = (int64_t)h[C_SAMPLES];
    s.fallback_rays = (int64_t)h[C_FALLBACK];
    s.shadow_fallback_rays = (int64_t)h[C_SFALLBACK];
    s.nee_vertices = (int64_t)h[C_NEEVTX];
    s.coop_overflows = (int64_t)h[C_COOPOVF];
#if RT_SIMD_STATS
    unsigned long long sm[8];
    simd_stats_read(sm);
    std::fprintf(stderr, "SIMD closest nodes %.3f tris %.3f | any nodes %.3f tris %.3f | steps %llu %llu %llu %llu\n",
                 sm[1] / (double)(sm[0] + !sm[0]), sm[3] / (double)(sm[2] + !sm[2]), sm[5] / (double)(sm[4] + !sm[4]),
                 sm[7] / (double)(sm[6] + !sm[6]), sm[0] / 64, sm[2] / 64, sm[4] / 64, sm[6] / 64);
#endif
    *out = s;
    return RT_OK;
}

static int reset_stats_one(rt_ctx* c) {
    if (!c) return RT_E_ARG;
    hipSetDevice(c->device);
    HIPCHK(c, hipDeviceSynchronize());
    harvest(c);
    c->stats = rt_stats{};
    HIPCHK(c, hipMemset(c->d_ctr, 0, sizeof(unsigned long long) * kCtrWords));
    return RT_OK;
}

static int impl_rt_octree_get_info(rt_ctx* c, rt_octree_info* out) {
    if (!c || !out) return RT_E_ARG;
    if (!c->have_scene) return fail(c, RT_E_STATE, "no scene");
    *out = c->info;
    return RT_OK;
}

static int impl_rt_octree_export(rt_ctx* c, float* bounds, int32_t* child, int32_t* leaf_first, int32_t* leaf_count, int32_t* refs) {
    if (!c) return RT_E_ARG;
    if (!c->have_scene) return fail(c, RT_E_STATE, "no scene");
    if (bounds) std::memcpy(bounds, c->h_bounds.data(), c->h_bounds.size() * 4);
    if (child) std::memcpy(child, c->h_child.data(), c->h_child.size() * 4);
    if (leaf_first) std::memcpy(leaf_first, c->h_leaf_first.data(), c->h_leaf_first.size() * 4);
    if (leaf_count) std::memcpy(leaf_count, c->h_leaf_count.data(), c->h_leaf_count.size() * 4);
    if (refs) std::memcpy(refs, c->h_refs.data(), c->h_refs.size() * 4);
    return RT_OK;
}

// The fast traversal's BVH as uploaded (tile set `set`): counts always, arrays when the pointers are non-null.
static int impl_rt_bvh_export(rt_ctx* c, int set, int* n_nodes, int* n_tiles, float* consts, float* nodes, float* tiles) {
    if (!c || set < 0 || set > 2) return RT_E_ARG;
    if (!c->have_scene) return fail(c, RT_E_STATE, "no scene");
    if (set == 1 && !c->cull) set = 0;  // the kernels use set 0's arrays when there is no culled set
    if (n_nodes) *n_nodes = c->bvh_count[set][0];
    if (n_tiles) *n_tiles = c->bvh_count[set][1];
    if (consts) { consts[0] = c->dsc.wabs; consts[1] = c->dsc.oguard; }
    hipSetDevice(c->device);
    if (nodes && c->bvh_count[set][0])
        HIPCHK(c, hipMemcpy(nodes, c->dsc.bvh[set], (size_t)c->bvh_count[set][0] * kBvhNodeF4 * 16, hipMemcpyDeviceToHost));
    if (tiles && c->bvh_count[set][1]) {  // the device's compact tiles + ids, exported in the 12-float view
        const int nt = c->bvh_count[set][1];
        std::vector<float> t9(9 * (size_t)nt);
        std::vector<int> tid(nt);
        HIPCHK(c, hipMemcpy(t9.data(), c->dsc.btiles[set], t9.size() * 4, hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(tid.data(), c->dsc.btid[set], tid.size() * 4, hipMemcpyDeviceToHost));
        bvh_tiles_logical(t9.data(), tid.data(), nt, tiles);
    }
    return RT_OK;
}

// The same BVH built on the host alone (no device): the upload's world transform, tile-set filter, padding and
// build parameters (RTMI_BVH_CI / RTMI_BVH_LEAF as rt_create reads them).  For CPU tests of the traversal.
static int impl_rt_debug_bvh_build(const rt_scene_desc* s, int set, int* n_nodes, int* n_tiles, float* consts,
                                   float* nodes, float* tiles) {
    if (!s || set < 0 || set > 2 || s->n_triangles <= 0 || s->n_vertices <= 0 || !s->positions || !s->indices)
        return RT_E_ARG;
    if (s->cull_backfaces && !s->normals) return RT_E_ARG;
    for (int t = 0; t < 3 * s->n_triangles; ++t)
        if (s->indices[t] >= (uint32_t)s->n_vertices) return RT_E_ARG;
    float cost = 2.5f;
    int leaf = kBvhMaxLeaf;
    if (const char* e = std::getenv("RTMI_BVH_CI")) cost = (float)std::atof(e);
    if (const char* e = std::getenv("RTMI_BVH_LEAF")) leaf = std::max(1, std::min(15, std::atoi(e)));
    if (set == kBvhAny) {  // rt_create's default (cost 2, leaves <= 4) / RTMI_BVH_ANY ("0/..": set 0's closest-hit BVH)
        float ac = 2.f;
        int al = 4;
        parse_bvh_any(ac, al);
        if (ac > 0) { cost = ac; leaf = al; }
    }
    SceneWorld sw;
    scene_world(s, sw);
    BvhData b;
    float wabs = 0.f, oguard = 0.f;
    scene_bvh(sw, set == 1 && s->cull_backfaces ? 1 : 0, cost, leaf, b, wabs, oguard);
    if (n_nodes) *n_nodes = (int)(b.nodes.size() / kBvhNodeF4);
    if (n_tiles) *n_tiles = (int)b.tid.size();
    if (consts) { consts[0] = wabs; consts[1] = oguard; }
    if (nodes) std::memcpy(nodes, b.nodes.data(), b.nodes.size() * 16);
    if (tiles) bvh_tiles_logical(b.tiles.data(), b.tid.data(), (int)b.tid.size(), tiles);
    return RT_OK;
}

static int impl_rt_debug_trace(rt_ctx* c, int n, const float* ro, const float* rd, int use_cull, int32_t* prim, float* bt) {
    if (!c || n < 0 || (n && (!ro || !rd || !prim || !bt))) return RT_E_ARG;
    if (!c->have_scene) return fail(c, RT_E_STATE, "no scene");
    if (n == 0) return RT_OK;
    hipSetDevice(c->device);
    std::vector<float4> o(n), d(n);
    for (int i = 0; i < n; ++i) {
        o[i] = make_float4(ro[3 * i], ro[3 * i + 1], ro[3 * i + 2], 0.f);
        d[i] = make_float4(rd[3 * i], rd[3 * i + 1], rd[3 * i + 2], 0.f);
    }
    float4 *dO = nullptr, *dD = nullptr, *dH = nullptr;
    int *dP = nullptr, *dT = nullptr, *dF = nullptr;
    // RTMI_DEBUG_PATH_KERNELS (multi-level scenes): the kernel path mode launches — wave tickets, the BVH walk, the
    // cooperative BFS for the undecided rays (or k_trace_fallback without coop_ok) — instead of the per-thread one
    const bool path_kernel = c->debug_path && c->dsc.qcap != 1;
    int rc = ensure_ring(c, c->ws[0]);
    if (!rc) rc = order_after_previous(c, c->stream);
    if (!rc && (dalloc(&dO, n) || dalloc(&dD, n) || dalloc(&dH, n) || dalloc(&dP, n) ||
                (path_kernel && (dalloc(&dT, 2 * kQStride) || dalloc(&dF, n)))))
        rc = fail(c, RT_E_OOM, "debug trace buffers");
    if (!rc) {
        TraceIO io{dO, dD, QueueView{nullptr, shard_stride(n, 1), n, 1}, (use_cull && c->cull) ? 1 : 0, dH, dP};
        if (path_kernel) {  // (ticket counter at dT[0], fallback list length at dT[kQStride])
            io.ticket = dT;
            io.fb_pos = dF;
            io.fb_len = dT + kQStride;
        }
        const DevScene& ls = lane_scene(c, c->ws[0]);
        if ((path_kernel && hipMemsetAsync(dT, 0, 2 * kQStride * sizeof(int), c->stream) != hipSuccess) ||
            hipMemcpy(dO, o.data(), 16 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(dD, d.data(), 16 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
            launch_trace_closest(c->stream, 0, c->dsc.qcap, ls, io, c->d_ctr) != hipSuccess ||
            (path_kernel && !c->dsc.coop_ok &&
             launch_trace_fallback(c->stream, 64, c->dsc.qcap, ls, io, c->d_ctr) != hipSuccess) ||
            hipStreamSynchronize(c->stream) != hipSuccess || hipMemcpy(prim, dP, 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(bt, dH, 16 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(c, RT_E_HIP, std::string("debug trace: ") + hipGetErrorString(hipGetLastError()));
    }
    hipFree(dO); hipFree(dD); hipFree(dH); hipFree(dP); hipFree(dT); hipFree(dF);
    if (!rc)
        for (int i = 0; i < n; ++i)
            if (prim[i] < 0) bt[4 * i] = bt[4 * i + 1] = bt[4 * i + 2] = bt[4 * i + 3] = 0.f;
    return rc;
}

static int impl_rt_debug_occluded(rt_ctx* c, int n, const float* ro, const float* rd, const float* tmax, int32_t* occluded) {
    if (!c || n < 0 || (n && (!ro || !rd || !tmax || !occluded))) return RT_E_ARG;
    if (!c->have_scene) return fail(c, RT_E_STATE, "no scene");
    if (n == 0) return RT_OK;
    hipSetDevice(c->device);
    std::vector<float4> o(n), d(n);
    for (int i = 0; i < n; ++i) {
        o[i] = make_float4(ro[3 * i], ro[3 * i + 1], ro[3 * i + 2], 0.f);
        d[i] = make_float4(rd[3 * i], rd[3 * i + 1], rd[3 * i + 2], tmax[i]);
    }
    float4 *dO = nullptr, *dD = nullptr;
    int* dP = nullptr;
    int rc = ensure_ring(c, c->ws[0]);
    if (!rc) rc = order_after_previous(c, c->stream);
    if (!rc && (dalloc(&dO, n) || dalloc(&dD, n) || dalloc(&dP, n))) rc = fail(c, RT_E_OOM, "debug occlusion buffers");
    if (!rc &&
        (hipMemcpy(dO, o.data(), 16 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(dD, d.data(), 16 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
         launch_occluded(c->stream, c->dsc.qcap, lane_scene(c, c->ws[0]), n, dO, dD, dP, c->d_ctr,
                         c->debug_path && c->dsc.coop_ok) != hipSuccess ||
         hipStreamSynchronize(c->stream) != hipSuccess ||
         hipMemcpy(occluded, dP, 4 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess))
        rc = fail(c, RT_E_HIP, std::string("debug occlusion: ") + hipGetErrorString(hipGetLastError()));
    hipFree(dO); hipFree(dD); hipFree(dP);
    return rc;
}

// The coherence sorts alone (rt_sort.hip) on a synthetic sharded queue: kShards shards of stride S, shard j holding
// shard_len[j] items at positions [j S, j S + shard_len[j]) with keys[pos] (and, for the NEE sort, slots[pos]).
// which 0: the ray sort (key bits 3 + 2 bits_a + 3 bits_b; out[pos'] = the queue position of sorted item pos'),
// 1: the NEE sort (key bits 3 bits_a; out = the slots sorted in place).  Sorted item k' sits at position
// (k' / S2) S + k' % S2 with S2 = shard_stride(n, kShards); out_len[j] receives the rewritten shard lengths.
static int impl_rt_debug_sort(rt_ctx* c, int which, int S, const int32_t* shard_len, const uint32_t* keys,
                              const int32_t* slots, int bits_a, int bits_b, int32_t* out, int32_t* out_len) {
    if (!c || (which != 0 && which != 1) || S < 64 || S % 64 || !shard_len || !keys || !out || !out_len ||
        (which == 1 && !slots))
        return c ? fail(c, RT_E_ARG, "debug sort: bad arguments") : RT_E_ARG;
    for (int j = 0; j < kShards; ++j)
        if (shard_len[j] < 0 || shard_len[j] > S) return fail(c, RT_E_ARG, "debug sort: shard length out of range");
    const int kb = which == 0 ? 3 + 2 * bits_a + 3 * bits_b : 3 * bits_a;
    if (bits_a < 0 || bits_a > (which == 0 ? 4 : 9) || bits_b < 0 || bits_b > 9 || kb < 1 || kb > 30)
        return fail(c, RT_E_ARG, "debug sort: key bits out of range");
    hipSetDevice(c->device);
    int rc = order_after_previous(c, c->stream);
    if (rc) return rc;
    const size_t cap = (size_t)kShards * S;
    unsigned *dkey = nullptr, *k0 = nullptr, *k1 = nullptr;
    int *dslot = nullptr, *dlen = nullptr, *dout = nullptr, *v0 = nullptr, *v1 = nullptr;
    void* temp = nullptr;
    if (dalloc(&dkey, cap) || dalloc(&dslot, cap) || dalloc(&dlen, (size_t)kShards * kQStride) || dalloc(&dout, cap) ||
        dalloc(&k0, cap) || dalloc(&k1, cap) || dalloc(&v0, cap) || dalloc(&v1, cap) ||
        hipMalloc(&temp, sort_temp_bytes()) != hipSuccess)
        rc = fail(c, RT_E_OOM, "debug sort buffers");
    if (!rc) {
        std::vector<int> hlen((size_t)kShards * kQStride, 0);
        for (int j = 0; j < kShards; ++j) hlen[(size_t)j * kQStride] = shard_len[j];
        std::vector<int> hs(cap, -1);
        if (which == 1) std::memcpy(hs.data(), slots, cap * 4);
        hipError_t e = hipMemcpy(dkey, keys, cap * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(dslot, hs.data(), cap * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(dlen, hlen.data(), hlen.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemset(dout, 0xff, cap * 4);
        if (e == hipSuccess) {
            if (which == 0) {
                SortRaysIO so{dkey, dout, k0, k1, v0, v1, temp, bits_a, bits_b, dlen, S};
                e = launch_sort_rays(c->stream, so);
            } else {
                SortNeeIO so{dslot, dlen, S, dkey, k0, k1, v0, v1, temp, bits_a};
                e = launch_sort_nee(c->stream, so);
            }
        }
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) e = hipMemcpy(out, which == 0 ? dout : dslot, cap * 4, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(hlen.data(), dlen, hlen.size() * 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = fail(c, RT_E_HIP, std::string("debug sort: ") + hipGetErrorString(e));
        else
            for (int j = 0; j < kShards; ++j) out_len[j] = hlen[(size_t)j * kQStride];
    }
    hipFree(dkey); hipFree(dslot); hipFree(dlen); hipFree(dout);
    hipFree(k0); hipFree(k1); hipFree(v0); hipFree(v1); hipFree(temp);
    if (!rc) rc = mark_done(c, c->stream);
    return rc;
}

static int impl_rt_debug_samples(rt_ctx* c, int n, const int32_t* pixel_ids, const int32_t* indices, rt_sample_record* out) {
    int rc = check_ready(c);
    if (rc) return rc;
    if (n < 0 || (n && (!pixel_ids || !indices || !out))) return fail(c, RT_E_ARG, "bad arguments");
    if (c->integ.kind != RT_INTEGRATOR_REFERENCE) return fail(c, RT_E_ARG, "records are for the reference integrator");
    if (n == 0) return RT_OK;
    int npx = c->film.res_x * c->film.res_y;
    if ((rc = ensure_sobol(c))) return rc;
    DevSampler smp = dev_sampler(c);
    for (int i = 0; i < n; ++i) {
        if (pixel_ids[i] < 0 || pixel_ids[i] >= npx || indices[i] < 0) return fail(c, RT_E_ARG, "sample out of range");
        if (c->smp.kind == RT_SAMPLER_STRATIFIED && !c->smp.jitter && indices[i] >= smp.spp)
            return fail(c, RT_E_ARG, "StratifiedSampler without jitter supports indices < SamplesPerPixel");
    }
    hipSetDevice(c->device);
    if ((rc = ensure_workspace(c, (size_t)n, false))) return rc;
    if ((rc = order_after_previous(c, c->stream))) return rc;
    int *dp = nullptr, *di = nullptr;
    float* dout = nullptr;
    static_assert(sizeof(rt_sample_record) == 39 * 4, "record layout");
    if (dalloc(&dp, n) || dalloc(&di, n) || dalloc(&dout, (size_t)n * 39)) rc = fail(c, RT_E_OOM, "record buffers");
    if (!rc) {
        hipMemcpy(dp, pixel_ids, 4 * (size_t)n, hipMemcpyHostToDevice);
        hipMemcpy(di, indices, 4 * (size_t)n, hipMemcpyHostToDevice);
        SampleIds ids{nullptr, 1, 0, dp, di};
        GenOut go{c->ws[0].rayO, c->ws[0].rayD, c->ws[0].lamA, c->ws[0].lamB, c->ws[0].pdfA,
                  c->ws[0].pdfB, RecView{nullptr, 0, 0}, 0, 1};
        DevFilm fd = dev_film(c);
        TraceIO tio{c->ws[0].rayO, c->ws[0].rayD, QueueView{nullptr, shard_stride(n, 1), n, 1}, c->cull ? 1 : 0, c->ws[0].hitB,
                    c->ws[0].hitPrim, nullptr, 1};
        ShadeRefIO sio = shade_ref_io(c);
        sio.rayD = c->ws[0].rayD; sio.lamA = c->ws[0].lamA; sio.lamB = c->ws[0].lamB; sio.pdfA = c->ws[0].pdfA; sio.pdfB = c->ws[0].pdfB;
        sio.hitB = c->ws[0].hitB; sio.hitPrim = c->ws[0].hitPrim;
        RecordIO rio{n, c->ws[0].rayO, c->ws[0].rayD, c->ws[0].lamA, c->ws[0].lamB, c->ws[0].pdfA, c->ws[0].pdfB, c->ws[0].hitB, c->ws[0].hitPrim, dout, 39, 1};
        if (launch_generate(c->stream, 0, n, ids, dev_camera(c->cam), smp, fd, go) != hipSuccess ||
            launch_trace_closest(c->stream, 0, c->dsc.qcap, lane_scene(c, c->ws[0]), tio, c->d_ctr) != hipSuccess ||
            launch_records(c->stream, c->dsc, c->d_spec, fd, sio, rio) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(out, dout, sizeof(rt_sample_record) * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(c, RT_E_HIP, std::string("debug samples: ") + hipGetErrorString(hipGetLastError()));
    }
    hipFree(dp); hipFree(di); hipFree(dout);
    return rc;
}

// ---- multi-device wrappers: configuration goes to every device of the context -------------------------------
extern "C++" template <class F>
static int on_all(rt_ctx* c, F f) {
    int rc = f(c);
    for (size_t j = 0; !rc && j < c->peers.size(); ++j) {
        rt_ctx* p = c->peers[j];
        hipSetDevice(p->device);
        if ((rc = f(p))) fail(c, rc, "device " + std::to_string(p->device) + ": " + p->err);
    }
    hipSetDevice(c->device);
    return rc;
}

static int impl_rt_create(const rt_options* opt, rt_ctx** out) {
    if (!out) return RT_E_ARG;
    *out = nullptr;
    int nd = opt ? opt->n_devices : 0;
    if (nd <= 1) return create_one(opt, out);
    if (nd > RT_MAX_DEVICES) return RT_E_ARG;
    rt_options o = *opt;
    o.n_devices = 0;
    o.device = opt->devices[0];
    rt_ctx* c = nullptr;
    int rc = create_one(&o, &c);
    if (rc) return rc;
    for (int j = 1; j < nd; ++j) {
        rt_ctx* p = nullptr;
        o.device = opt->devices[j];
        if ((rc = create_one(&o, &p))) { rt_destroy(c); return rc; }
        c->peers.push_back(p);
        c->links.emplace_back();
        if (p->device != c->device) {  // direct xGMI peer copies both ways where the platform allows them
            int ok = 0;
            if (hipDeviceCanAccessPeer(&ok, c->device, p->device) == hipSuccess && ok) {
                hipSetDevice(c->device);
                if (hipDeviceEnablePeerAccess(p->device, 0) != hipSuccess) (void)hipGetLastError();
                hipSetDevice(p->device);
                if (hipDeviceEnablePeerAccess(c->device, 0) != hipSuccess) (void)hipGetLastError();
            }
        }
        hipSetDevice(p->device);
        if (hipEventCreateWithFlags(&p->gathered, hipEventDisableTiming) != hipSuccess) { rt_destroy(c); return RT_E_HIP; }
    }
    hipSetDevice(c->device);
    if (hipEventCreateWithFlags(&c->gathered, hipEventDisableTiming) != hipSuccess) { rt_destroy(c); return RT_E_HIP; }
    if ((rc = rt_set_shard(c, 32, 1, 0))) { rt_destroy(c); return rc; }
    *out = c;
    return RT_OK;
}

static void impl_rt_destroy(rt_ctx* c) {
    if (!c) return;
    for (size_t j = 0; j < c->peers.size(); ++j) {
        rt_ctx* p = c->peers[j];
        hipSetDevice(p->device);
        if (p->stream) hipStreamSynchronize(p->stream);
        if (p->xfer) hipFree(p->xfer);
        if (p->gathered) hipEventDestroy(p->gathered);
        destroy_one(p);
    }
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    for (rt_ctx::PeerLink& L : c->links) {
        if (L.work0) hipFree(L.work0);
        if (L.xfer0) hipFree(L.xfer0);
    }
    if (c->gathered) hipEventDestroy(c->gathered);
    destroy_one(c);
}

static int impl_rt_scene_upload(rt_ctx* c, const rt_scene_desc* s) {
    if (!c) return RT_E_ARG;
    return on_all(c, [&](rt_ctx* x) { return scene_upload_one(x, s); });
}
static int impl_rt_camera_set(rt_ctx* c, const rt_camera_desc* d) {
    if (!c) return RT_E_ARG;
    return on_all(c, [&](rt_ctx* x) { return camera_set_one(x, d); });
}
static int impl_rt_sampler_set(rt_ctx* c, const rt_sampler_desc* d) {
    if (!c) return RT_E_ARG;
    return on_all(c, [&](rt_ctx* x) { return sampler_set_one(x, d); });
}
static int impl_rt_film_set(rt_ctx* c, const rt_film_desc* d) {
    if (!c) return RT_E_ARG;
    return on_all(c, [&](rt_ctx* x) { return film_set_one(x, d); });
}
static int impl_rt_integrator_set(rt_ctx* c, const rt_integrator_desc* d) {
    if (!c) return RT_E_ARG;
    return on_all(c, [&](rt_ctx* x) { return integrator_set_one(x, d); });
}
static int impl_rt_reset_stats(rt_ctx* c) {
    if (!c) return RT_E_ARG;
    return on_all(c, [&](rt_ctx* x) { return reset_stats_one(x); });
}
// the caller's shard (tile t, t % n_shards == shard_id) is split over the context's D devices: device k takes the
// tiles with (t / n_shards) % D == k, i.e. shard (n_shards·D, shard_id + n_shards·k) of the frame
// counters and kernel times summed over the context's devices
static int impl_rt_get_stats(rt_ctx* c, rt_stats* out) {
    if (!c || !out) return RT_E_ARG;
    rt_stats sum{};
    int rc = on_all(c, [&](rt_ctx* x) -> int {
        rt_stats s{};
        int r = get_stats_one(x, &s);
        if (r) return r;
        sum.samples += s.samples; sum.rays += s.rays; sum.shadow_rays += s.shadow_rays;
        sum.nodes_tested += s.nodes_tested; sum.tris_tested += s.tris_tested; sum.hits += s.hits;
        sum.shadow_nodes_tested += s.shadow_nodes_tested; sum.shadow_tris_tested += s.shadow_tris_tested;
        sum.ms_generate += s.ms_generate; sum.ms_trace += s.ms_trace; sum.ms_shade += s.ms_shade;
        sum.ms_shadow += s.ms_shadow; sum.ms_film += s.ms_film; sum.ms_sort += s.ms_sort;
        sum.launches_trace += s.launches_trace; sum.launches_shade += s.launches_shade;
        sum.fallback_rays += s.fallback_rays; sum.shadow_fallback_rays += s.shadow_fallback_rays;
        sum.nee_vertices += s.nee_vertices;
        sum.coop_overflows += s.coop_overflows;
        return RT_OK;
    });
    if (!rc) *out = sum;
    return rc;
}

static int impl_rt_set_shard(rt_ctx* c, int tile_size, int n_shards, int shard_id) {
    if (!c || n_shards <= 0 || shard_id < 0 || shard_id >= n_shards)
        return c ? fail(c, RT_E_ARG, "invalid shard") : RT_E_ARG;
    const int D = 1 + (int)c->peers.size();
    int rc = set_shard_one(c, tile_size, n_shards * D, shard_id);
    for (size_t j = 0; !rc && j < c->peers.size(); ++j)
        if ((rc = set_shard_one(c->peers[j], tile_size, n_shards * D, shard_id + n_shards * (int)(j + 1))))
            fail(c, rc, c->peers[j]->err);
    return rc;
}

}  // extern "C"

// ---- the exception firewall around every entry point (rt_guard.h)
extern "C" {
int rt_film_matrices(rt_ctx* c, float* xyz_from_sensor9, float* rgb_from_xyz9) {
    return guarded([&] { return impl_rt_film_matrices(c, xyz_from_sensor9, rgb_from_xyz9); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_render_pass_device(rt_ctx* c, int ib, int ie, void* d_film, void* stream) {
    return guarded([&] { return impl_rt_render_pass_device(c, ib, ie, d_film, stream); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_render_pass(rt_ctx* c, int ib, int ie, rt_pixel* film) {
    return guarded([&] { return impl_rt_render_pass(c, ib, ie, film); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_film_resolve(rt_ctx* c, const rt_pixel* film, uint8_t* out) {
    return guarded([&] { return impl_rt_film_resolve(c, film, out); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_film_resolve_srgb(rt_ctx* c, const rt_pixel* film, uint8_t* out) {
    return guarded([&] { return impl_rt_film_resolve_srgb(c, film, out); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_octree_get_info(rt_ctx* c, rt_octree_info* out) {
    return guarded([&] { return impl_rt_octree_get_info(c, out); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_octree_export(rt_ctx* c, float* bounds, int32_t* child, int32_t* leaf_first, int32_t* leaf_count, int32_t* refs) {
    return guarded([&] { return impl_rt_octree_export(c, bounds, child, leaf_first, leaf_count, refs); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_bvh_export(rt_ctx* c, int set, int* n_nodes, int* n_tiles, float* consts, float* nodes, float* tiles) {
    return guarded([&] { return impl_rt_bvh_export(c, set, n_nodes, n_tiles, consts, nodes, tiles); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_debug_bvh_build(const rt_scene_desc* s, int set, int* n_nodes, int* n_tiles, float* consts, float* nodes, float* tiles) {
    return guarded([&] { return impl_rt_debug_bvh_build(s, set, n_nodes, n_tiles, consts, nodes, tiles); }, [](const std::string&) {});
}
int rt_debug_trace(rt_ctx* c, int n, const float* ro, const float* rd, int use_cull, int32_t* prim, float* bt) {
    return guarded([&] { return impl_rt_debug_trace(c, n, ro, rd, use_cull, prim, bt); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_debug_occluded(rt_ctx* c, int n, const float* ro, const float* rd, const float* tmax, int32_t* occluded) {
    return guarded([&] { return impl_rt_debug_occluded(c, n, ro, rd, tmax, occluded); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_debug_samples(rt_ctx* c, int n, const int32_t* pixel_ids, const int32_t* indices, rt_sample_record* out) {
    return guarded([&] { return impl_rt_debug_samples(c, n, pixel_ids, indices, out); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_debug_sort(rt_ctx* c, int which, int S, const int32_t* shard_len, const uint32_t* keys, const int32_t* slots,
                  int bits_a, int bits_b, int32_t* out, int32_t* out_len) {
    return guarded([&] { return impl_rt_debug_sort(c, which, S, shard_len, keys, slots, bits_a, bits_b, out, out_len); },
                   [&](const std::string& m) { set_error(c, m); });
}
int rt_create(const rt_options* opt, rt_ctx** out) {
    return guarded([&] { return impl_rt_create(opt, out); }, [&](const std::string& m) { set_error(nullptr, m); });
}
int rt_scene_upload(rt_ctx* c, const rt_scene_desc* s) {
    return guarded([&] { return impl_rt_scene_upload(c, s); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_camera_set(rt_ctx* c, const rt_camera_desc* d) {
    return guarded([&] { return impl_rt_camera_set(c, d); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_sampler_set(rt_ctx* c, const rt_sampler_desc* d) {
    return guarded([&] { return impl_rt_sampler_set(c, d); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_film_set(rt_ctx* c, const rt_film_desc* d) {
    return guarded([&] { return impl_rt_film_set(c, d); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_integrator_set(rt_ctx* c, const rt_integrator_desc* d) {
    return guarded([&] { return impl_rt_integrator_set(c, d); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_reset_stats(rt_ctx* c) {
    return guarded([&] { return impl_rt_reset_stats(c); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_get_stats(rt_ctx* c, rt_stats* out) {
    return guarded([&] { return impl_rt_get_stats(c, out); }, [&](const std::string& m) { set_error(c, m); });
}
int rt_set_shard(rt_ctx* c, int tile_size, int n_shards, int shard_id) {
    return guarded([&] { return impl_rt_set_shard(c, tile_size, n_shards, shard_id); }, [&](const std::string& m) { set_error(c, m); });
}
void rt_destroy(rt_ctx* c) {
    guarded([&] { impl_rt_destroy(c); return 0; }, [](const std::string&) {}, /*inject=*/false);
}

}  // extern "C"
