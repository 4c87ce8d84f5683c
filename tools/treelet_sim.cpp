// Treelet-queue cost model for the multi-level closest-hit walk.
//
// Walks rays over the product's 8-wide BVH (the rt_bvh.cpp layout, as rt_debug_bvh_build exports it) with the kernels'
// node order (nearest child first, far children pushed, entries beyond the cut dropped on pop, cut = t1 + 2 W(t1)) and
// counts, per ray, the node visits, triangle tests and how often the walk crosses from one treelet to another, for a
// partition of the tree into treelets of at most B bytes (80 B per node as the kernels read it + 36 B per triangle
// tile): the subtree of a node is one treelet when it fits B, the nodes above those roots form the top treelet 0.
// A treelet-queue traversal moves a ray's state through HBM once per crossing, so crossings per ray price it.
// Measurement tool only (analysis input: tools/treelet_sim.py); the triangle test is a plain float Möller-Trumbore,
// which decides the same hits as the watertight test up to rounding — enough for visit counts.
//
//   g++ -O2 -std=c++17 -o tools/_build/treelet_sim tools/treelet_sim.cpp
//   treelet_sim nodes.f32 n_nodes tiles.f32 n_tiles rays.f32 n_rays wabs B1 [B2 ...]  > stats
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static uint32_t U(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static float F(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

struct Bvh {
    std::vector<float> nodes, tiles;  // 32 floats per node, 12 per tile
    int nn = 0, nt = 0;
    const float* N(int i) const { return nodes.data() + 32 * (size_t)i; }
    void keys(int node, const float inv[3], const float oi[3], float tcut, unsigned k[8]) const {
        const float* n = N(node);
        const uint32_t w0 = U(n[3]), valid = U(n[7]);
        float s[3], b[3];
        for (int a = 0; a < 3; ++a) {
            s[a] = std::ldexp(inv[a], (int)((w0 >> (8 * a)) & 255u) - 127);
            b[a] = std::fma(n[a], inv[a], -oi[a]);
        }
        for (int sl = 0; sl < 8; ++sl) {
            float tn = 0.f, tf = tcut;
            for (int a = 0; a < 3; ++a) {
                const float* q = n + 8 + 4 * a;
                const uint32_t lo = (U(q[sl >> 2]) >> (8 * (sl & 3))) & 255u, hi = (U(q[2 + (sl >> 2)]) >> (8 * (sl & 3))) & 255u;
                const bool pos = inv[a] >= 0.f;
                tn = std::fmax(tn, std::fma((float)(pos ? lo : hi), s[a], b[a]));
                tf = std::fmin(tf, std::fma((float)(pos ? hi : lo), s[a], b[a]));
            }
            tf *= 1.00000048f;
            k[sl] = (((valid >> sl) & 1u) && tn <= tf) ? ((U(tn) & 0x7ffffff8u) | (unsigned)sl) : 0xffffffffu;
        }
        std::sort(k, k + 8);
    }
    int word(int node, unsigned key) const {
        const float* n = N(node);
        const unsigned s = key & 7u, imask = U(n[3]) >> 24;
        if ((imask >> s) & 1u) return (int)(U(n[4]) + (unsigned)__builtin_popcount(imask & ((1u << s) - 1u)));
        const unsigned counts = U(n[6]), cnt = (counts >> (4 * s)) & 15u;
        unsigned first = U(n[5]);
        for (unsigned j = 0; j < s; ++j) first += (counts >> (4 * j)) & 15u;
        return (int)(0x80000000u | first << 4 | (cnt - 1u));
    }
    // children of a node: internal node ids and leaf tile ranges
    void children(int node, std::vector<int>& in, std::vector<std::pair<int, int>>& lv) const {
        const float* n = N(node);
        const uint32_t valid = U(n[7]);
        for (int s = 0; s < 8; ++s) {
            if (!((valid >> s) & 1u)) continue;
            const int w = word(node, (unsigned)s);
            if (w >= 0) in.push_back(w);
            else lv.emplace_back((w >> 4) & 0x7ffffff, (w & 15) + 1);
        }
    }
};

static bool moller(const float* q, const float o[3], const float d[3], float tmax, float& t) {
    const float e1[3] = {q[3] - q[0], q[4] - q[1], q[5] - q[2]}, e2[3] = {q[6] - q[0], q[7] - q[1], q[8] - q[2]};
    const float p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
    const float det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    if (det == 0.f) return false;
    const float id = 1.f / det;
    const float s[3] = {o[0] - q[0], o[1] - q[1], o[2] - q[2]};
    const float u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) * id;
    if (u < 0.f || u > 1.f) return false;
    const float qq[3] = {s[1] * e1[2] - s[2] * e1[1], s[2] * e1[0] - s[0] * e1[2], s[0] * e1[1] - s[1] * e1[0]};
    const float v = (d[0] * qq[0] + d[1] * qq[1] + d[2] * qq[2]) * id;
    if (v < 0.f || u + v > 1.f) return false;
    t = (e2[0] * qq[0] + e2[1] * qq[1] + e2[2] * qq[2]) * id;
    return t > 0.f && t < tmax;
}

static std::vector<float> readf(const char* path, size_t n) {
    std::vector<float> v(n);
    FILE* f = std::fopen(path, "rb");
    if (!f || std::fread(v.data(), 4, n, f) != n) { std::fprintf(stderr, "read %s\n", path); std::exit(1); }
    std::fclose(f);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 9) { std::fprintf(stderr, "usage: see header\n"); return 2; }
    Bvh bvh;
    bvh.nn = std::atoi(argv[2]);
    bvh.nt = std::atoi(argv[4]);
    const int nr = std::atoi(argv[6]);
    const float wabs = (float)std::atof(argv[7]);
    bvh.nodes = readf(argv[1], 32 * (size_t)bvh.nn);
    bvh.tiles = readf(argv[3], 12 * (size_t)bvh.nt);
    const std::vector<float> rays = readf(argv[5], 6 * (size_t)nr);  // o.xyz, d.xyz per ray (sorted order)
    // subtree bytes (80 B per node read, 36 B per tile) bottom-up: children have larger ids than their parent
    // except the breadth-first top levels, so iterate to a fixed point
    std::vector<double> sub(bvh.nn, 0.0);
    std::vector<std::vector<int>> kids(bvh.nn);
    std::vector<int> ntiles(bvh.nn, 0);
    for (int i = 0; i < bvh.nn; ++i) {
        std::vector<std::pair<int, int>> lv;
        bvh.children(i, kids[i], lv);
        for (auto& l : lv) ntiles[i] += l.second;
    }
    std::vector<int> order;  // post-order from the root
    {
        std::vector<std::pair<int, int>> st{{0, 0}};
        while (!st.empty()) {
            auto& [n, c] = st.back();
            if (c < (int)kids[n].size()) { const int ch = kids[n][c++]; st.push_back({ch, 0}); }
            else { order.push_back(n); st.pop_back(); }
        }
    }
    for (int n : order) {
        sub[n] = 80.0 + 36.0 * ntiles[n];
        for (int c : kids[n]) sub[n] += sub[c];
    }
    std::printf("nodes %d tiles %d tree_bytes %.0f rays %d\n", bvh.nn, bvh.nt, sub[0], nr);
    for (int ai = 8; ai < argc; ++ai) {
        const double B = std::atof(argv[ai]);
        // treelet of every node: roots = highest nodes whose subtree fits B; the rest is the top (treelet 0)
        std::vector<int> tl(bvh.nn, 0);
        int ntl = 1;
        double top_bytes = 0;
        std::vector<int> st{0};
        while (!st.empty()) {
            const int n = st.back();
            st.pop_back();
            if (sub[n] <= B) {
                const int id = ntl++;
                std::vector<int> s2{n};
                while (!s2.empty()) { const int m = s2.back(); s2.pop_back(); tl[m] = id; for (int c : kids[m]) s2.push_back(c); }
            } else {
                tl[n] = 0;
                top_bytes += 80.0 + 36.0 * ntiles[n];
                for (int c : kids[n]) st.push_back(c);
            }
        }
        long long visits = 0, tris = 0, cross = 0, distinct = 0, wave_distinct = 0, waves = 0, nodes_top = 0;
        std::vector<int> wave_set;
        for (int r = 0; r < nr; ++r) {
            const float* R = rays.data() + 6 * (size_t)r;
            const float o[3] = {R[0], R[1], R[2]}, d[3] = {R[3], R[4], R[5]};
            float inv[3], oi[3];
            for (int a = 0; a < 3; ++a) {
                inv[a] = 1 / std::copysign(std::max(std::fabs(d[a]), 0x1p-80f), d[a]);
                oi[a] = o[a] * inv[a];
            }
            float cut = 3.4e38f, t1 = 3.4e38f;
            struct E { int w; unsigned key; int parent; };
            std::vector<E> stk;
            std::vector<int> seen;
            int cur_tl = -1;
            auto enter = [&](int t) {
                if (t != cur_tl) { if (cur_tl >= 0) ++cross; cur_tl = t; }
                if (std::find(seen.begin(), seen.end(), t) == seen.end()) seen.push_back(t);
                if (std::find(wave_set.begin(), wave_set.end(), t) == wave_set.end()) wave_set.push_back(t);
            };
            int node = 0;
            while (true) {
                int lf = 0, lc = 0;
                while (lc == 0) {
                    if (node < 0) {
                        if (stk.empty()) break;
                        auto e = stk.back();
                        stk.pop_back();
                        if (F(e.key & 0x7ffffff8u) > cut) continue;
                        const int w = e.w;
                        if (w >= 0) node = w;
                        else { lf = (w >> 4) & 0x7ffffff; lc = (w & 15) + 1; enter(tl[e.parent]); }  // its tiles
                        continue;
                    }
                    ++visits;
                    if (tl[node] == 0) ++nodes_top;
                    enter(tl[node]);
                    unsigned k[8];
                    bvh.keys(node, inv, oi, cut, k);
                    const int c = node;
                    node = -1;
                    for (int i = 7; i >= 1; --i)
                        if (k[i] != 0xffffffffu) stk.push_back(E{bvh.word(c, k[i]), k[i], c});
                    if (k[0] != 0xffffffffu) {
                        const int w = bvh.word(c, k[0]);
                        if (w >= 0) node = w;
                        else { lf = (w >> 4) & 0x7ffffff; lc = (w & 15) + 1; }
                    }
                }
                if (lc == 0) break;
                for (int k = 0; k < lc; ++k) {
                    ++tris;
                    float t;
                    if (moller(bvh.tiles.data() + 12 * (size_t)(lf + k), o, d, cut, t) && t < t1) {
                        t1 = t;
                        cut = std::min(cut, t + 2.f * (t * 0x1p-16f + wabs));
                    }
                }
            }
            distinct += (long long)seen.size();
            if ((r & 63) == 63 || r == nr - 1) { wave_distinct += (long long)wave_set.size(); ++waves; wave_set.clear(); }
        }
        std::printf("B %.0f treelets %d top_bytes %.0f | per ray: visits %.2f top_visits %.2f tris %.2f crossings %.2f "
                    "distinct_treelets %.2f | per 64-ray wave: distinct treelets %.1f\n",
                    B, ntl, top_bytes, visits / (double)nr, nodes_top / (double)nr, tris / (double)nr,
                    cross / (double)nr, distinct / (double)nr, wave_distinct / (double)waves);
    }
    return 0;
}
