// 8-wide compressed BVH over a tile set's triangles (host build, uploaded with the scene) for the fast multi-level
// traversal of rt_kernels.hip.  The BVH never decides a result on its own: the kernels apply the
// canonical closest-hit / any-hit rule over the triangles it reaches and hand every ambiguous ray to the
// reference-order octree BFS (Octtree_Model.h:66-127), so only the set of triangles reachable by a ray matters,
// and every box is rounded outwards (conservative: a triangle the watertight test hits at t lies in boxes the ray
// enters before t).
//
// Build: binned SAH (64 bins per axis, leaves of <= kMaxLeaf triangles) into a binary tree, collapsed to 8-wide
// nodes by an SAH-optimal dynamic program over the binary tree (round 4; round 3 opened the largest-area internal
// child until there were 8: CFG3 9,314 -> 5,918 wide nodes, node visits per bounce ray 4.69 -> 4.54).
//
// Node (one 128-B cache line, 8 float4; the kernels read the first five):
//   N0 = (origin.xyz, bits: ex | ey << 8 | ez << 16 | imask << 24)   origin = the node's padded box corner,
//        e_a = the biased exponent of the axis' quantum 2^(e_a - 127); imask bit k = child slot k is a node
//   N1 = (child_base, tile_base, counts, valid)   internal child k = child_base + popcount(imask below k); leaf
//        child k = counts nibble k triangles (1..15) at tile_base + the sum of the nibbles below k; valid bit k =
//        slot k is used
//   N2..N4 = the x, y, z child planes: u8 lo[8] then u8 hi[8] per axis; the child's box along a is
//        [origin_a + lo 2^(e_a-127), origin_a + hi 2^(e_a-127)] ⊇ its triangles' box padded by `pad` (exact:
//        lo = floor, hi = ceil of the exact quotients, computed in double)
//   N5..N7 = zero (line padding)
// The top of the tree is laid out breadth-first at the front (every node with an id below kBvhTopNodes has its
// children block reserved in breadth-first order; those nodes are staged in LDS by the kernels), every deeper subtree
// depth-first after them: a node's internal children are one contiguous block,
// its leaf children's tiles one contiguous run, in the same depth-first order as the nodes (treelet-contiguous).
// Tiles (compact, round 4): 9 floats (36 B) per triangle, p0.xyz p1.xyz p2.xyz, packed back to back in leaf order, and
// the triangle id of each tile in a parallel int array (read once per ray, for the winning tile only).  The octree
// tiles' 48-B format (p0.xyz, p1.x) (p1.yz, p2.xy) (p2.z, bits(id), 0, 0) remains the exported, logical view
// (bvh_tiles_logical): CFG3's closest-hit tiles shrink from 4.7 MB to 3.5 MB + 0.4 MB of ids.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "rt_internal.h"

namespace rtmi {
namespace {

struct Box {
    float lo[3], hi[3];
    Box() {
        for (int a = 0; a < 3; ++a) { lo[a] = std::numeric_limits<float>::infinity(); hi[a] = -lo[a]; }
    }
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
    }
    void grow(const float* p) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], p[a]); hi[a] = std::max(hi[a], p[a]); }
    }
    double area() const {
        double e[3];
        for (int a = 0; a < 3; ++a) e[a] = hi[a] >= lo[a] ? (double)hi[a] - lo[a] : 0.0;
        return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
    }
};

struct Node2 {
    Box box;
    int left = -1, right = -1;  // internal: children; leaf: left = -1
    int first = 0, count = 0;   // leaf range in the permutation
};

constexpr int kBins = 64;  // (r04: 16 -> 64 bins: CFG3 bounce rays 5.45 -> 4.70 node visits per ray, tools/bvh_quality.py)

struct Builder {
    float node_cost = 1.f;       // SAH: cost of opening a node relative to one triangle test
    int max_leaf = kBvhMaxLeaf;
    std::vector<Box> pbox;
    std::vector<float> cen;      // 3 per primitive
    std::vector<int> perm;
    std::vector<Node2> nodes;

    int build(int b, int e) {
        const int id = (int)nodes.size();
        nodes.emplace_back();
        Box bb, cb;
        for (int i = b; i < e; ++i) {
            bb.grow(pbox[perm[i]]);
            cb.grow(&cen[3 * (size_t)perm[i]]);
        }
        nodes[id].box = bb;
        const int n = e - b;
        if (n <= 2 && n <= max_leaf) {
            nodes[id].first = b; nodes[id].count = n;
            return id;
        }
        // best binned SAH split over the three centroid axes
        double best = std::numeric_limits<double>::infinity();
        int bax = -1, bsplit = 0;
        for (int a = 0; a < 3; ++a) {
            const float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0)) continue;
            Box bin[kBins];
            int cnt[kBins] = {0};
            const float k = (float)kBins / ext;
            for (int i = b; i < e; ++i) {
                int j = (int)((cen[3 * (size_t)perm[i] + a] - cb.lo[a]) * k);
                j = std::min(std::max(j, 0), kBins - 1);
                ++cnt[j];
                bin[j].grow(pbox[perm[i]]);
            }
            double ra[kBins];
            int rn[kBins];
            Box acc;
            int c = 0;
            for (int j = kBins - 1; j > 0; --j) {
                acc.grow(bin[j]); c += cnt[j];
                ra[j] = acc.area(); rn[j] = c;
            }
            Box lacc;
            int lc = 0;
            for (int j = 1; j < kBins; ++j) {
                lacc.grow(bin[j - 1]); lc += cnt[j - 1];
                if (lc == 0 || rn[j] == 0) continue;
                const double cost = lacc.area() * lc + ra[j] * rn[j];
                if (cost < best) { best = cost; bax = a; bsplit = j; }
            }
        }
        const double parea = std::max(bb.area(), 1e-30);
        const double split_cost = node_cost + best / parea;
        if (n <= max_leaf && (bax < 0 || (double)n <= split_cost)) {
            nodes[id].first = b; nodes[id].count = n;
            return id;
        }
        int mid;
        if (bax < 0) {  // coincident centroids: split by count
            mid = b + n / 2;
        } else {
            const float k = (float)kBins / (cb.hi[bax] - cb.lo[bax]);
            auto it = std::partition(perm.begin() + b, perm.begin() + e, [&](int p) {
                int j = (int)((cen[3 * (size_t)p + bax] - cb.lo[bax]) * k);
                j = std::min(std::max(j, 0), kBins - 1);
                return j < bsplit;
            });
            mid = (int)(it - perm.begin());
            if (mid == b || mid == e) mid = b + n / 2;
        }
        const int l = build(b, mid);
        const int r = build(mid, e);
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }
};

struct Collapse {
    const Builder& B;
    const float* tri9;
    const int* ids;
    double pad;
    BvhData& out;
    int depth_max = 0;

    // Which binary nodes become the children of each 8-wide node: an SAH-optimal collapse (dynamic programming over
    // the binary tree, Ylitie et al. 2017).  C1[n] = the cost of binary node n as one child of a wide node (a leaf:
    // area x triangles; an internal node: a wide node of its own, area x wide_cost + its best spread D[n][8]);
    // D[n][k] = the least cost of n's two subtrees spread over at most k child slots (each subtree either one child,
    // C1, or opened again); Ck(n, k) = min(C1[n], D[n][k]).  Costs are areas: the SAH's hit probabilities.
    double wide_cost = 3.0;  // a wide node's visit relative to one triangle test (1-12: the same CFG3 / CFG4 trees)
    std::vector<double> C1;
    std::vector<std::array<double, 9>> D;
    std::vector<std::array<int, 9>> Dsplit;  // D[n][k]'s slots for the left subtree
    double Ck(int n, int k) const { return k <= 1 || B.nodes[n].left < 0 ? C1[n] : std::min(C1[n], D[n][k]); }
    void plan(int root) {
        const size_t nn = B.nodes.size();
        C1.assign(nn, 0.0);
        D.assign(nn, {});
        Dsplit.assign(nn, {});
        // children have larger indices than their parent (pre-order build): a reverse sweep is post-order
        for (size_t i = nn; i-- > 0;) {
            const Node2& x = B.nodes[i];
            const double a = x.box.area();
            if (x.left < 0) {
                C1[i] = a * x.count;
                continue;
            }
            for (int k = 2; k <= 8; ++k) {
                double best = std::numeric_limits<double>::infinity();
                int bs = 1;
                for (int kl = 1; kl < k; ++kl) {
                    const double c = Ck(x.left, kl) + Ck(x.right, k - kl);
                    if (c < best) { best = c; bs = kl; }
                }
                D[i][k] = best;
                Dsplit[i][k] = bs;
            }
            C1[i] = a * wide_cost + D[i][8];
        }
        (void)root;
    }
    void expand(int n, int k, std::vector<int>& ch) const {
        if (k <= 1 || B.nodes[n].left < 0 || C1[n] <= D[n][k]) {
            ch.push_back(n);
            return;
        }
        const int kl = Dsplit[n][k];
        expand(B.nodes[n].left, kl, ch);
        expand(B.nodes[n].right, k - kl, ch);
    }
    // the up-to-8 binary nodes that become the children of the 8-wide node for binary node n2
    std::vector<int> children8(int n2) const {
        std::vector<int> ch;
        if (B.nodes[n2].left < 0) {
            ch.push_back(n2);  // a leaf root
            return ch;
        }
        const int kl = Dsplit[n2][8];
        expand(B.nodes[n2].left, kl, ch);
        expand(B.nodes[n2].right, 8 - kl, ch);
        return ch;
    }
    int reserve(int n) {
        const int me = (int)(out.nodes.size() / kBvhNodeF4);
        out.nodes.resize(out.nodes.size() + (size_t)n * kBvhNodeF4, make_float4(0.f, 0.f, 0.f, 0.f));
        return me;
    }
    int n_internal(const std::vector<int>& ch) const {
        int k = 0;
        for (int c : ch) k += B.nodes[c].left >= 0;
        return k;
    }
    // Quantise the children of node `me` (binary ids ch, slot order) and write its header.  Internal children
    // are the nodes child_base, child_base + 1, ... in slot order; leaf children's tiles are appended here.
    void write_node(int me, const std::vector<int>& ch, int child_base) {
        double lo[8][3], hi[8][3];
        double plo[3] = {INFINITY, INFINITY, INFINITY}, phi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = 0; k < ch.size(); ++k) {
            const Box& b = B.nodes[ch[k]].box;
            for (int a = 0; a < 3; ++a) {
                lo[k][a] = (double)b.lo[a] - pad;
                hi[k][a] = (double)b.hi[a] + pad;
                plo[a] = std::min(plo[a], lo[k][a]);
                phi[a] = std::max(phi[a], hi[k][a]);
            }
        }
        float org[3];
        int ebias[3];
        for (int a = 0; a < 3; ++a) {
            // the float origin at or below the padded corner, then the smallest quantum 2^e with 255 2^e >= extent
            float o = (float)plo[a];
            if ((double)o > plo[a]) o = std::nextafter(o, -INFINITY);
            org[a] = o;
            const double ext = phi[a] - (double)o;
            int e = -100;
            if (ext > 0) {
                e = (int)std::ceil(std::log2(ext / 255.0));
                while (std::ldexp(255.0, e) < ext) ++e;
                while (e > -100 && std::ldexp(255.0, e - 1) >= ext) --e;
            }
            ebias[a] = e + 127;
        }
        unsigned qlo[3][8] = {}, qhi[3][8] = {};
        unsigned imask = 0, valid = 0, counts = 0;
        const int tile_base = (int)out.tid.size();
        int ci = 0;
        for (size_t k = 0; k < ch.size(); ++k) {
            const Node2& c = B.nodes[ch[k]];
            for (int a = 0; a < 3; ++a) {
                const double q = std::ldexp(1.0, ebias[a] - 127);
                const double l = std::floor((lo[k][a] - (double)org[a]) / q);
                const double h = std::ceil((hi[k][a] - (double)org[a]) / q);
                qlo[a][k] = (unsigned)std::min(std::max(l, 0.0), 255.0);
                qhi[a][k] = (unsigned)std::min(std::max(h, 0.0), 255.0);
            }
            valid |= 1u << k;
            if (c.left >= 0) {
                imask |= 1u << k;
                ++ci;
            } else {
                counts |= (unsigned)c.count << (4 * k);
                for (int i = c.first; i < c.first + c.count; ++i) {
                    const int p = B.perm[i];
                    const float* v = tri9 + 9 * (size_t)p;
                    out.tiles.insert(out.tiles.end(), v, v + 9);
                    out.tid.push_back(ids[p]);
                }
                out.max_leaf = std::max(out.max_leaf, c.count);
            }
        }
        (void)ci;
        float4* nd = &out.nodes[(size_t)kBvhNodeF4 * me];
        unsigned w0 = (unsigned)ebias[0] | (unsigned)ebias[1] << 8 | (unsigned)ebias[2] << 16 | imask << 24;
        float fw0;
        std::memcpy(&fw0, &w0, 4);
        nd[0] = make_float4(org[0], org[1], org[2], fw0);
        const unsigned h1[4] = {(unsigned)child_base, (unsigned)tile_base, counts, valid};
        std::memcpy(&nd[1], h1, 16);
        for (int a = 0; a < 3; ++a) {
            unsigned w[4] = {0, 0, 0, 0};
            for (int k = 0; k < 8; ++k) {
                w[k >> 2] |= qlo[a][k] << (8 * (k & 3));
                w[2 + (k >> 2)] |= qhi[a][k] << (8 * (k & 3));
            }
            std::memcpy(&nd[2 + a], w, 16);  // the bytes' bits, never through float registers
        }
    }
    // depth-first: node `me` for binary node n2, its children block, then each internal child's subtree
    void emit(int n2, int me, int depth) {
        depth_max = std::max(depth_max, depth);
        const std::vector<int> ch = children8(n2);
        const int ni = n_internal(ch);
        const int base = ni ? reserve(ni) : 0;
        write_node(me, ch, base);
        int k = 0;
        for (int c : ch)
            if (B.nodes[c].left >= 0) emit(c, base + k++, depth + 1);
    }
    // breadth-first while the node's id is below kBvhTopNodes (the nodes staged in LDS by the kernels), every node
    // after that depth-first (9 nodes: the root and its children; 73: three full levels)
    void emit_root(int root) {
        struct Item { int n2, me, depth; };
        std::vector<Item> fifo{{root, reserve(1), 0}};
        size_t h = 0;
        for (; h < fifo.size() && fifo[h].me < kBvhTopNodes; ++h) {
            const Item it = fifo[h];
            depth_max = std::max(depth_max, it.depth);
            const std::vector<int> ch = children8(it.n2);
            const int ni = n_internal(ch);
            const int base = ni ? reserve(ni) : 0;
            write_node(it.me, ch, base);
            int k = 0;
            for (int c : ch)
                if (B.nodes[c].left >= 0) fifo.push_back({c, base + k++, it.depth + 1});
        }
        for (; h < fifo.size(); ++h) emit(fifo[h].n2, fifo[h].me, fifo[h].depth);
    }
};

}  // namespace

void build_bvh8(const float* tri9, const int* ids, int n, float pad, float node_cost, BvhData& out, int max_leaf) {
    out.nodes.clear();
    out.tiles.clear();
    out.tid.clear();
    out.max_leaf = 0;
    out.depth = 0;
    if (n == 0) {  // an empty root: no valid child
        out.nodes.assign(kBvhNodeF4, make_float4(0.f, 0.f, 0.f, 0.f));
        return;
    }
    Builder B;
    B.node_cost = node_cost;
    B.max_leaf = std::min(std::max(max_leaf, 1), 15);
    B.pbox.resize(n);
    B.cen.resize(3 * (size_t)n);
    B.perm.resize(n);
    for (int i = 0; i < n; ++i) {
        Box b;
        for (int v = 0; v < 3; ++v) b.grow(tri9 + 9 * (size_t)i + 3 * v);
        B.pbox[i] = b;
        for (int a = 0; a < 3; ++a) B.cen[3 * (size_t)i + a] = 0.5f * (b.lo[a] + b.hi[a]);
        B.perm[i] = i;
    }
    B.nodes.reserve(2 * (size_t)n);
    B.build(0, n);
    Collapse C{B, tri9, ids, (double)pad, out};
    C.plan(0);
    out.nodes.reserve((size_t)kBvhNodeF4 * (n / 4 + 1));
    out.tiles.reserve(9 * (size_t)n);
    out.tid.reserve((size_t)n);
    C.emit_root(0);
    out.depth = C.depth_max;
}

void bvh_tiles_logical(const float* t9, const int* tid, int n, float* out12) {
    for (int i = 0; i < n; ++i) {
        float* o = out12 + 12 * (size_t)i;
        std::memcpy(o, t9 + 9 * (size_t)i, 9 * sizeof(float));
        std::memcpy(o + 9, &tid[i], 4);
        o[10] = o[11] = 0.f;
    }
}

}  // namespace rtmi
