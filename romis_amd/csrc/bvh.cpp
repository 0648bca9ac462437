// bvh.cpp -- binned-SAH BVH over the scene triangles, flattened to the threaded (miss-link) layout.
//
// The tree only prunes: every candidate triangle is still decided by the exact Moller-Trumbore test, so the
// BVH shape never changes a result (DESIGN.md "Visibility").  Box bounds are padded by a small scene-relative
// margin to keep the device slab test conservative under rounding.
#include "bvh.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

namespace romis {
namespace {

struct Box {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    float hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(const float* p) {
        for (int a = 0; a < 3; a++) { lo[a] = std::min(lo[a], p[a]); hi[a] = std::max(hi[a], p[a]); }
    }
    void grow(const Box& b) {
        for (int a = 0; a < 3; a++) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
    }
    float area() const {
        float d[3];
        for (int a = 0; a < 3; a++) d[a] = std::max(0.0f, hi[a] - lo[a]);
        return 2.0f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

struct TmpNode {
    Box box;
    int left = -1, right = -1;
    uint32_t first = 0, count = 0;
};

struct Builder {
    const std::vector<BvhTriangle>& tris;
    std::vector<Box> tbox;
    std::vector<float> cent;   // [T][3]
    std::vector<uint32_t> idx;
    std::vector<TmpNode> nodes;
    uint32_t max_leaf;
    uint32_t max_depth = 0;

    explicit Builder(const std::vector<BvhTriangle>& t, uint32_t ml) : tris(t), max_leaf(ml) {
        const size_t T = t.size();
        tbox.resize(T);
        cent.resize(3 * T);
        idx.resize(T);
        for (size_t i = 0; i < T; i++) {
            tbox[i].grow(t[i].v0); tbox[i].grow(t[i].v1); tbox[i].grow(t[i].v2);
            for (int a = 0; a < 3; a++) cent[3 * i + a] = 0.5f * (tbox[i].lo[a] + tbox[i].hi[a]);
            idx[i] = (uint32_t)i;
        }
    }

    int build(uint32_t first, uint32_t count, uint32_t depth) {
        max_depth = std::max(max_depth, depth);
        int id = (int)nodes.size();
        nodes.emplace_back();
        Box b, cb;
        for (uint32_t i = first; i < first + count; i++) { b.grow(tbox[idx[i]]); cb.grow(&cent[3 * idx[i]]); }
        nodes[id].box = b;
        if (count <= max_leaf) { nodes[id].first = first; nodes[id].count = count; return id; }

        // binned SAH over the centroid bounds, 16 bins per axis
        constexpr int NB = 16;
        float best_cost = FLT_MAX;
        int best_axis = -1, best_split = -1;
        for (int a = 0; a < 3; a++) {
            float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.0f)) continue;
            Box bins[NB];
            uint32_t cnt[NB] = {0};
            for (uint32_t i = first; i < first + count; i++) {
                int k = std::min(NB - 1, (int)((cent[3 * idx[i] + a] - cb.lo[a]) / ext * NB));
                bins[k].grow(tbox[idx[i]]);
                cnt[k]++;
            }
            float la[NB], ra[NB];
            uint32_t lc[NB], rc[NB];
            Box acc;
            uint32_t c = 0;
            for (int k = 0; k < NB; k++) { acc.grow(bins[k]); c += cnt[k]; la[k] = acc.area(); lc[k] = c; }
            acc = Box();
            c = 0;
            for (int k = NB - 1; k >= 0; k--) { acc.grow(bins[k]); c += cnt[k]; ra[k] = acc.area(); rc[k] = c; }
            for (int k = 0; k < NB - 1; k++) {
                if (lc[k] == 0 || rc[k + 1] == 0) continue;
                float cost = la[k] * lc[k] + ra[k + 1] * rc[k + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = k; }
            }
        }
        uint32_t mid;
        if (best_axis < 0) {
            mid = first + count / 2;   // all centroids coincide: split the range in half
        } else {
            const float ext = cb.hi[best_axis] - cb.lo[best_axis];
            auto it = std::stable_partition(idx.begin() + first, idx.begin() + first + count, [&](uint32_t t) {
                int k = std::min(NB - 1, (int)((cent[3 * t + best_axis] - cb.lo[best_axis]) / ext * NB));
                return k <= best_split;
            });
            mid = (uint32_t)(it - idx.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        int l = build(first, mid - first, depth + 1);
        int r = build(mid, first + count - mid, depth + 1);
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }
};

uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

}  // namespace

FlatBvh build_bvh(const std::vector<BvhTriangle>& tris, uint32_t max_leaf) {
    FlatBvh out;
    if (tris.empty()) return out;
    max_leaf = std::min<uint32_t>(std::max<uint32_t>(max_leaf, 1u), 255u);
    Builder b(tris, max_leaf);
    b.build(0, (uint32_t)tris.size(), 0);
    out.max_depth = b.max_depth;

    // scene-relative padding
    const Box& root = b.nodes[0].box;
    float scale = 0.0f;
    for (int a = 0; a < 3; a++) scale = std::max({scale, std::fabs(root.lo[a]), std::fabs(root.hi[a]), root.hi[a] - root.lo[a]});
    const float pad = 1e-5f * scale + 1e-30f;

    // preorder flatten: subtree sizes give right-child indices; miss(left) = right, miss(right) = miss(parent)
    const size_t n = b.nodes.size();
    std::vector<uint32_t> pre(n), size(n);
    // iterative post-order for sizes
    std::vector<int> stack{0}, order;
    while (!stack.empty()) {
        int v = stack.back(); stack.pop_back();
        order.push_back(v);
        if (b.nodes[v].left >= 0) { stack.push_back(b.nodes[v].left); stack.push_back(b.nodes[v].right); }
    }
    for (auto it = order.rbegin(); it != order.rend(); ++it) {
        int v = *it;
        size[v] = 1;
        if (b.nodes[v].left >= 0) size[v] += size[b.nodes[v].left] + size[b.nodes[v].right];
    }
    out.num_nodes = (uint32_t)n;
    out.nodes.assign(8 * n, 0.0f);
    struct Item { int v; uint32_t index; uint32_t miss; };
    std::vector<Item> st{{0, 0u, (uint32_t)n}};
    while (!st.empty()) {
        Item it = st.back(); st.pop_back();
        const TmpNode& nd = b.nodes[it.v];
        float* o = &out.nodes[8 * it.index];
        for (int a = 0; a < 3; a++) { o[a] = nd.box.lo[a] - pad; o[4 + a] = nd.box.hi[a] + pad; }
        o[3] = u2f(it.miss);
        if (nd.left < 0) {
            o[7] = u2f((nd.count << 24) | nd.first);
        } else {
            o[7] = u2f(0u);
            uint32_t li = it.index + 1, ri = it.index + 1 + size[nd.left];
            st.push_back({nd.right, ri, it.miss});
            st.push_back({nd.left, li, ri});
        }
    }
    out.tri_order = b.idx;
    return out;
}

}  // namespace romis
