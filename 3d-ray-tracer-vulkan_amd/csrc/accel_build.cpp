// accel_build.cpp — option "accel": a binned-SAH tree over the reference's
// triangles, in near-first preorder layouts (accel_build.h).
//
// Inputs are the reference's own buffers (SceneBuilder.java:92-104,
// BVHFlattener.java:51-97).  Each leaf of the reference tree names a flattened
// triangle and holds that triangle's box (Triangle.calculateBoundingBox,
// Triangle.java:61-71: the double box with +1e-4 on flat axes, cast to
// float); that (triangle, box) pair is one primitive here.  The reference
// flattens a node of one triangle into two leaves of the same triangle
// (BVHBuilder.java:60-62), so about a third of the flattened triangles are
// copies of their predecessor: a primitive whose vertices, material and box are
// byte-identical to one with a lower flattened index is dropped (the copy
// can never be the closest hit: same t, higher index).
//
// The tree: binned SAH (32 bins per axis over the primitive box centroids,
// cost = area x count on each side), one primitive per leaf; an internal
// node's box is the union of its children's (exact in float).  Node ids are
// implicit (a subtree of m primitives takes 2m - 1 nodes and 3m - 1 slots),
// so subtrees build on several threads and the result does not depend on the
// thread count.
#include "accel_build.h"

#include <algorithm>
#include <cstring>
#include <thread>

namespace rtamd {

namespace {

struct Prim {
    float lo[3], hi[3];
    float c[3];       // box centroid
    int tri;          // flattened triangle index
};

struct BNode {
    float lo[3], hi[3];
    int axis = 0;     // split axis (internal)
    int prim = -1;    // >= 0: a leaf of this primitive
    int m = 0;        // primitives in the subtree
    int left = -1, right = -1;   // node ids (internal): lower-centroid side first
};

constexpr int kBins = 32;

float area(const float lo[3], const float hi[3]) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

struct Builder {
    std::vector<Prim> prims;
    std::vector<int> ids;
    std::vector<BNode> nodes;
    unsigned max_threads = 1;

    // Builds the subtree of ids[b, e) as node `id` (its descendants take ids
    // id + 1 .. id + 2m - 2); returns its depth below id.
    int build(int id, int b, int e, unsigned threads) {
        BNode& nd = nodes[id];
        const int m = e - b;
        nd.m = m;
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = prims[ids[b]].lo[k];
            nd.hi[k] = prims[ids[b]].hi[k];
        }
        for (int i = b + 1; i < e; ++i)
            for (int k = 0; k < 3; ++k) {
                nd.lo[k] = std::min(nd.lo[k], prims[ids[i]].lo[k]);
                nd.hi[k] = std::max(nd.hi[k], prims[ids[i]].hi[k]);
            }
        if (m == 1) {
            nd.prim = ids[b];
            return 0;
        }
        // centroid bounds
        float clo[3], chi[3];
        for (int k = 0; k < 3; ++k) clo[k] = chi[k] = prims[ids[b]].c[k];
        for (int i = b + 1; i < e; ++i)
            for (int k = 0; k < 3; ++k) {
                clo[k] = std::min(clo[k], prims[ids[i]].c[k]);
                chi[k] = std::max(chi[k], prims[ids[i]].c[k]);
            }
        int best_axis = -1, best_bin = -1;
        float best_cost = 0.0f;
        for (int k = 0; k < 3; ++k) {
            const float ext = chi[k] - clo[k];
            if (!(ext > 0.0f)) continue;
            const float scale = (float)kBins / ext;
            int cnt[kBins] = {};
            float blo[kBins][3], bhi[kBins][3];
            for (int j = 0; j < kBins; ++j)
                for (int q = 0; q < 3; ++q) {
                    blo[j][q] = INFINITY;
                    bhi[j][q] = -INFINITY;
                }
            for (int i = b; i < e; ++i) {
                const Prim& p = prims[ids[i]];
                const int j = std::min(kBins - 1, std::max(0, (int)((p.c[k] - clo[k]) * scale)));
                ++cnt[j];
                for (int q = 0; q < 3; ++q) {
                    blo[j][q] = std::min(blo[j][q], p.lo[q]);
                    bhi[j][q] = std::max(bhi[j][q], p.hi[q]);
                }
            }
            // right-to-left sweep: area x count of bins j.. ; then left to right
            float ra[kBins];
            int rc[kBins];
            float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int c = 0;
            for (int j = kBins - 1; j > 0; --j) {
                c += cnt[j];
                for (int q = 0; q < 3; ++q) {
                    lo[q] = std::min(lo[q], blo[j][q]);
                    hi[q] = std::max(hi[q], bhi[j][q]);
                }
                rc[j] = c;
                ra[j] = c ? area(lo, hi) : 0.0f;
            }
            for (int q = 0; q < 3; ++q) {
                lo[q] = INFINITY;
                hi[q] = -INFINITY;
            }
            c = 0;
            for (int j = 0; j < kBins - 1; ++j) {      // split between bins j and j + 1
                c += cnt[j];
                for (int q = 0; q < 3; ++q) {
                    lo[q] = std::min(lo[q], blo[j][q]);
                    hi[q] = std::max(hi[q], bhi[j][q]);
                }
                if (c == 0 || rc[j + 1] == 0) continue;
                const float cost = (float)c * area(lo, hi) + (float)rc[j + 1] * ra[j + 1];
                if (best_axis < 0 || cost < best_cost) {
                    best_axis = k;
                    best_bin = j;
                    best_cost = cost;
                }
            }
        }
        int mid;
        if (best_axis >= 0) {
            const int k = best_axis;
            const float scale = (float)kBins / (chi[k] - clo[k]);
            auto left_of = [&](int pi) {
                return std::min(kBins - 1, std::max(0, (int)((prims[pi].c[k] - clo[k]) * scale))) <= best_bin;
            };
            mid = (int)(std::stable_partition(ids.begin() + b, ids.begin() + e, left_of) - ids.begin());
            nd.axis = k;
        } else {
            // every centroid equal: halve in index order
            mid = b + m / 2;
            nd.axis = 0;
        }
        if (mid <= b || mid >= e) mid = b + m / 2;
        const int ml = mid - b;
        nd.left = id + 1;
        nd.right = id + 2 * ml;   // id + 1 + (2 ml - 1)
        int dl, dr;
        if (threads > 1 && m > 16384) {
            std::thread th([&] { dl = build(id + 1, b, mid, threads / 2); });
            dr = build(id + 2 * ml, mid, e, threads - threads / 2);
            th.join();
        } else {
            dl = build(id + 1, b, mid, 1);
            dr = build(id + 2 * ml, mid, e, 1);
        }
        return 1 + std::max(dl, dr);
    }
};

uint64_t fnv(const unsigned char* p, size_t n, uint64_t h) {
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

void put_f(uint32_t* w, float f) { std::memcpy(w, &f, 4); }

}  // namespace

int accel_build(const void* vertices, size_t vertex_bytes, const void* materials, size_t material_bytes,
                const void* bvh_nodes, size_t bvh_bytes, int n_layouts, int n_threads, AccelHost* out,
                std::string* err) {
    *out = AccelHost{};
    if (n_layouts != 1 && n_layouts != 8) {
        *err = "accel: n_layouts must be 1 or 8";
        return -1;
    }
    out->n_layouts = n_layouts;
    const size_t n_nodes = bvh_bytes / 48, n_tris = vertex_bytes / 48, n_mats = material_bytes / 16;
    const unsigned char* nb = static_cast<const unsigned char*>(bvh_nodes);
    const unsigned char* vb = static_cast<const unsigned char*>(vertices);
    const unsigned char* mb = static_cast<const unsigned char*>(materials);
    if (n_nodes == 0) {           // empty scene: no slots (two of padding), every ray misses
        out->rec.assign(16, 0u);
        return 0;
    }

    // 1. the reference's leaves as primitives (triangle, leaf box), duplicates dropped
    Builder B;
    struct Occ { uint64_t h; int tri; size_t node; };
    std::vector<Occ> occ;
    for (size_t k = 0; k < n_nodes; ++k) {
        int32_t data, count;
        std::memcpy(&data, nb + k * 48 + 32, 4);
        std::memcpy(&count, nb + k * 48 + 36, 4);
        if (count >= 0) continue;
        const int64_t tri = -((int64_t)data + 1);
        if (tri < 0 || (size_t)tri >= n_tris || (size_t)tri >= n_mats || tri >= (1 << 29)) {
            *err = "accel: leaf " + std::to_string(k) + " names triangle " + std::to_string(tri) +
                   " outside the buffers";
            return -1;
        }
        uint64_t h = fnv(vb + (size_t)tri * 48, 48, 1469598103934665603ull);
        h = fnv(mb + (size_t)tri * 16, 16, h);
        h = fnv(nb + k * 48, 12, h);
        h = fnv(nb + k * 48 + 16, 12, h);
        occ.push_back({h, (int)tri, k});
    }
    out->n_inputs = (int)occ.size();
    std::vector<int> order(occ.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int x, int y) {
        return occ[x].h != occ[y].h ? occ[x].h < occ[y].h : occ[x].tri < occ[y].tri;
    });
    std::vector<uint8_t> dup(occ.size(), 0);
    auto same = [&](const Occ& a, const Occ& b) {
        return std::memcmp(vb + (size_t)a.tri * 48, vb + (size_t)b.tri * 48, 48) == 0 &&
               std::memcmp(mb + (size_t)a.tri * 16, mb + (size_t)b.tri * 16, 16) == 0 &&
               std::memcmp(nb + a.node * 48, nb + b.node * 48, 12) == 0 &&
               std::memcmp(nb + a.node * 48 + 16, nb + b.node * 48 + 16, 12) == 0;
    };
    for (size_t s = 0; s < order.size();) {
        size_t e = s;
        while (e < order.size() && occ[order[e]].h == occ[order[s]].h) ++e;
        for (size_t i = s + 1; i < e; ++i)          // the group is in flattened-index order
            for (size_t j = s; j < i; ++j)
                if (!dup[order[j]] && same(occ[order[i]], occ[order[j]])) {
                    dup[order[i]] = 1;
                    break;
                }
        s = e;
    }
    for (size_t i = 0; i < occ.size(); ++i) {
        if (dup[i]) continue;
        Prim p;
        for (int q = 0; q < 3; ++q) {
            std::memcpy(&p.lo[q], nb + occ[i].node * 48 + 4 * q, 4);
            std::memcpy(&p.hi[q], nb + occ[i].node * 48 + 16 + 4 * q, 4);
            p.c[q] = 0.5f * (p.lo[q] + p.hi[q]);
        }
        p.tri = occ[i].tri;
        B.prims.push_back(p);
    }
    const int m = (int)B.prims.size();
    out->n_prims = m;
    const int64_t slots = 3 * (int64_t)m - 1;
    if (slots * n_layouts + 2 > (int64_t)((1u << 27) - 4)) {
        *err = "accel: " + std::to_string(m) + " triangles: the layouts exceed 2^27 slots (4 GB)";
        return -1;
    }

    // 2. the tree
    B.ids.resize(m);
    for (int i = 0; i < m; ++i) B.ids[i] = i;
    B.nodes.resize(2 * (size_t)m - 1);
    const unsigned hw = n_threads > 0 ? (unsigned)n_threads : std::max(1u, std::thread::hardware_concurrency());
    out->depth = B.build(0, 0, m, std::min(hw, 64u));
    {
        const float a0 = area(B.nodes[0].lo, B.nodes[0].hi);
        double s = 0.0;
        for (const BNode& nd : B.nodes) s += a0 > 0.0f ? (double)area(nd.lo, nd.hi) / a0 : 1.0;
        out->sah = s;
    }

    // 3. the layouts: preorder, near child first per the layout's sign bits
    out->slots = (int)slots;
    out->root_leaf = B.nodes[0].prim >= 0 ? 1 : 0;
    const size_t total = (size_t)slots * (size_t)n_layouts;
    out->rec.assign(8 * (total + 2), 0u);
    std::vector<uint8_t> leaf_at(total + 1, 0);
    for (int o = 0; o < n_layouts; ++o) {
        const size_t base = (size_t)o * (size_t)slots;
        struct Item { int node; size_t pos; };
        std::vector<Item> st;
        st.push_back({0, base});
        while (!st.empty()) {
            const Item it = st.back();
            st.pop_back();
            const BNode& nd = B.nodes[it.node];
            uint32_t* w = &out->rec[8 * it.pos];
            for (int q = 0; q < 3; ++q) {
                put_f(&w[q], nd.lo[q]);
                put_f(&w[4 + q], nd.hi[q]);
            }
            if (nd.prim >= 0) {
                leaf_at[it.pos] = 1;
                const Prim& p = B.prims[nd.prim];
                const unsigned char* v = vb + (size_t)p.tri * 48;
                float x[9];
                for (int j = 0; j < 3; ++j) std::memcpy(&x[3 * j], v + 16 * j, 12);
                // e1 = v1 - v0, e2 = v2 - v0, as hit_triangle computes them (:106-107)
                const float e1[3] = {x[3] - x[0], x[4] - x[1], x[5] - x[2]};
                const float e2[3] = {x[6] - x[0], x[7] - x[1], x[8] - x[2]};
                w[3] = (uint32_t)p.tri | (1u << 30);            // | L(next) << 31, below
                put_f(&w[7], x[0]);
                put_f(&w[8], x[1]);
                put_f(&w[9], x[2]);
                put_f(&w[10], e1[0]);
                put_f(&w[11], e1[1]);
                put_f(&w[12], e1[2]);
                put_f(&w[13], e2[0]);
                put_f(&w[14], e2[1]);
                put_f(&w[15], e2[2]);
                continue;
            }
            const bool neg = n_layouts == 8 && ((o >> nd.axis) & 1);
            const int first = neg ? nd.right : nd.left, second = neg ? nd.left : nd.right;
            const size_t skip = it.pos + 3 * (size_t)nd.m - 1;
            w[3] = (uint32_t)skip;                                 // | L(skip) << 31, below
            const size_t pos2 = it.pos + 1 + 3 * (size_t)B.nodes[first].m - 1;
            st.push_back({second, pos2});
            st.push_back({first, it.pos + 1});
        }
        // the L bits: an internal node's skip and first child, a leaf's successor
        const size_t end = base + (size_t)slots;
        auto L = [&](size_t s) -> uint32_t { return s < end && leaf_at[s] ? 1u : 0u; };
        for (size_t s = base; s < end;) {
            uint32_t* w = &out->rec[8 * s];
            if (leaf_at[s]) {
                w[3] |= L(s + 2) << 31;
                s += 2;
            } else {
                w[3] |= L(w[3]) << 31;
                w[7] = L(s + 1);
                s += 1;
            }
        }
    }
    return 0;
}

}  // namespace rtamd
