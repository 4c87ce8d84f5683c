// 4-wide BVH over a tile set's triangles (host build, uploaded with the scene) for the fast multi-level
// traversal of rt_kernels.hip.  The BVH never decides a result on its own: the kernels apply the
// canonical closest-hit / any-hit rule over the triangles it reaches and hand every ambiguous ray to the
// reference-order octree BFS (Octtree_Model.h:66-127), so only the set of triangles reachable by a ray matters,
// and every box is padded outwards (conservative: a triangle the watertight test hits at t lies in boxes the ray
// enters before t).
//
// Build: binned SAH (16 bins per axis, leaves of <= 8 triangles) into a binary tree, collapsed to 4-wide nodes by
// repeatedly opening the largest-area internal child.  Node layout (128 B, one cache line): float4 lo.x[4],
// hi.x[4], lo.y[4], hi.y[4], lo.z[4], hi.z[4], int4 child[4], pad.  Child words: >= 0 internal node, -1 empty,
// otherwise a leaf 0x80000000 | first_tile << 4 | (count - 1) over the leaf-ordered tile array (3 float4 per
// triangle, the octree tiles' format).
#include <algorithm>
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

constexpr int kBins = 16;
constexpr int kMaxLeaf = 8;

struct Builder {
    const float* tri9;
    float node_cost = 1.f;       // SAH: cost of opening a node relative to one triangle test
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
        if (n <= 2) {
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
        if (bax < 0 || (n <= kMaxLeaf && (double)n <= split_cost)) {
            if (n <= kMaxLeaf) {
                nodes[id].first = b; nodes[id].count = n;
                return id;
            }
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
    float pad;
    BvhData& out;
    int depth_max = 0;

    void push_tiles(const Node2& lf) {
        for (int i = lf.first; i < lf.first + lf.count; ++i) {
            const int p = B.perm[i];
            const float* v = tri9 + 9 * (size_t)p;
            float fid;
            std::memcpy(&fid, &ids[p], 4);
            out.tiles.push_back(make_float4(v[0], v[1], v[2], v[3]));
            out.tiles.push_back(make_float4(v[4], v[5], v[6], v[7]));
            out.tiles.push_back(make_float4(v[8], fid, 0.f, 0.f));
        }
    }
    int leaf_word(const Node2& lf) {
        const int first = (int)(out.tiles.size() / 3);
        push_tiles(lf);
        out.max_leaf = std::max(out.max_leaf, lf.count);
        return (int)(0x80000000u | ((unsigned)first << 4) | (unsigned)(lf.count - 1));
    }
    // the up-to-4 binary nodes that become the children of the 4-wide node for binary node n2 (opening the
    // largest-area internal child until there are 4)
    std::vector<int> children4(int n2) const {
        std::vector<int> ch;
        if (B.nodes[n2].left < 0) {
            ch.push_back(n2);  // a leaf root
            return ch;
        }
        ch = {B.nodes[n2].left, B.nodes[n2].right};
        while (ch.size() < 4) {
            int pick = -1;
            double pa = -1;
            for (size_t k = 0; k < ch.size(); ++k)
                if (B.nodes[ch[k]].left >= 0 && B.nodes[ch[k]].box.area() > pa) { pa = B.nodes[ch[k]].box.area(); pick = (int)k; }
            if (pick < 0) break;
            const int o = ch[pick];
            ch[pick] = B.nodes[o].left;
            ch.push_back(B.nodes[o].right);
        }
        return ch;
    }
    int reserve() {
        const int me = (int)(out.nodes.size() / 8);
        out.nodes.resize(out.nodes.size() + 8);
        return me;
    }
    void write_node(int me, const std::vector<int>& ch, const int* word) {
        float lo[3][4], hi[3][4];
        for (int k = 0; k < 4; ++k)
            for (int a = 0; a < 3; ++a) { lo[a][k] = 0.f; hi[a][k] = 0.f; }
        int w[4] = {-1, -1, -1, -1};
        for (size_t k = 0; k < ch.size(); ++k) {
            const Node2& c = B.nodes[ch[k]];
            for (int a = 0; a < 3; ++a) { lo[a][k] = c.box.lo[a] - pad; hi[a][k] = c.box.hi[a] + pad; }
            w[k] = word[k];
        }
        float4* nd = &out.nodes[8 * (size_t)me];
        for (int a = 0; a < 3; ++a) {
            nd[2 * a] = make_float4(lo[a][0], lo[a][1], lo[a][2], lo[a][3]);
            nd[2 * a + 1] = make_float4(hi[a][0], hi[a][1], hi[a][2], hi[a][3]);
        }
        std::memcpy(&nd[6], w, 16);  // the child words' bits, never through float registers
        nd[7] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // depth-first: the 4-wide node for binary node n2 and its subtree, appended; returns its index
    int emit(int n2, int depth) {
        depth_max = std::max(depth_max, depth);
        const int me = reserve();
        const std::vector<int> ch = children4(n2);
        int word[4] = {-1, -1, -1, -1};
        for (size_t k = 0; k < ch.size(); ++k)
            word[k] = B.nodes[ch[k]].left < 0 ? leaf_word(B.nodes[ch[k]]) : emit(ch[k], depth + 1);
        write_node(me, ch, word);
        return me;
    }
    // the top kBvhTopLevels levels breadth-first (nodes 0 .. kBvhTopNodes - 1 at most, which the kernels stage in
    // LDS), every deeper subtree depth-first after them
    void emit_root(int root) {
        std::vector<std::pair<int, int>> level = {{root, reserve()}};
        for (int depth = 0; depth < kBvhTopLevels && !level.empty(); ++depth) {
            depth_max = std::max(depth_max, depth);
            std::vector<std::pair<int, int>> next;
            std::vector<std::pair<int, std::vector<int>>> pend;  // (node index, children) of this level
            for (const auto& [n2, me] : level) {
                std::vector<int> ch = children4(n2);
                pend.emplace_back(me, ch);
            }
            // indices of the next level first (contiguous), then leaves / deeper subtrees
            std::vector<std::vector<int>> words(pend.size(), std::vector<int>(4, -1));
            for (size_t i = 0; i < pend.size(); ++i)
                for (size_t k = 0; k < pend[i].second.size(); ++k) {
                    const int c = pend[i].second[k];
                    if (B.nodes[c].left >= 0 && depth + 1 < kBvhTopLevels) {
                        words[i][k] = reserve();
                        next.emplace_back(c, words[i][k]);
                    }
                }
            for (size_t i = 0; i < pend.size(); ++i) {
                for (size_t k = 0; k < pend[i].second.size(); ++k) {
                    const int c = pend[i].second[k];
                    if (B.nodes[c].left < 0) words[i][k] = leaf_word(B.nodes[c]);
                    else if (depth + 1 >= kBvhTopLevels) words[i][k] = emit(c, depth + 1);
                }
                write_node(pend[i].first, pend[i].second, words[i].data());
            }
            level = std::move(next);
        }
    }
};

}  // namespace

void build_bvh4(const float* tri9, const int* ids, int n, float pad, float node_cost, BvhData& out) {
    out.nodes.clear();
    out.tiles.clear();
    out.max_leaf = 0;
    out.depth = 0;
    if (n == 0) {  // an empty root: every child word -1
        out.nodes.assign(8, make_float4(0.f, 0.f, 0.f, 0.f));
        float m1;
        const int neg = -1;
        std::memcpy(&m1, &neg, 4);
        out.nodes[6] = make_float4(m1, m1, m1, m1);
        return;
    }
    Builder B;
    B.tri9 = tri9;
    B.node_cost = node_cost;
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
    Collapse C{B, tri9, ids, pad, out};
    out.nodes.reserve(8 * (size_t)(n / 2 + 1));
    out.tiles.reserve(3 * (size_t)n);
    C.emit_root(0);
    out.depth = C.depth_max;
}

}  // namespace rtmi
