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
// The tree: full-sweep SAH (every object boundary of the box-centroid order
// on each axis, cost = area x count on each side; 32 bins measured 7.65 /
// 12.02 / 15.23 node visits per segment on configs 3 / 6 / 5 against 6.02 /
// 7.14 / 13.73 for the sweep, tools/accel_study.py), one primitive per leaf;
// an internal node's box is the union of its children's (exact in float).
// Node ids are implicit (a subtree of m primitives takes 2m - 1 nodes and
// 3m - 1 slots), so subtrees build on several threads and the result does not
// depend on the thread count.
#include "accel_build.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#ifdef ACCEL_TIMING
#include <chrono>
#include <cstdio>
#define ACCEL_T(msg) std::fprintf(stderr, "accel_build %s %.3f s\n", msg, std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count())
#else
#define ACCEL_T(msg)
#endif

namespace rtamd {

namespace {

struct Prim {
    float lo[3], hi[3];
    float c[3];       // box centroid
    int tri;          // flattened triangle index
    int cls;          // shape class (accel_class)
};

struct BNode {
    float lo[3], hi[3];
    int axis = 0;     // split axis (internal)
    int prim = -1;    // >= 0: a leaf of this primitive
    int m = 0;        // primitives in the subtree
    int left = -1, right = -1;   // node ids (internal): lower-centroid side first
    int cls = 0;      // the largest shape class in the subtree
};

float area(const float lo[3], const float hi[3]) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

// Full-sweep SAH over three presorted lists: ord[k] holds the primitives in
// the order of their box centroids on axis k (ties by primitive index).  A
// subtree owns the same range [b, e) of all three lists; a node tries every
// object boundary of every axis (cost = area x count on each side), and the
// chosen split partitions the other two lists stably, so every range stays
// sorted.  O(n log n) to sort, then O(n) per tree level.
struct Builder {
    std::vector<Prim> prims;
    std::vector<int> ord[3];
    std::vector<BNode> nodes;
    std::vector<uint8_t> left;      // scratch: primitive goes to the left child
    std::vector<int> tmp;           // scratch: stable partition
    std::vector<float> rarea;       // scratch: right-side areas

    // Below this depth a node splits at the median of its widest centroid
    // axis instead of by SAH: primitives whose boxes and centroids coincide
    // (copies of a triangle in other materials, nested boxes about one
    // centre) make every SAH split peel one primitive off, a tree m deep
    // built in O(m^2).  Ordinary scenes never get near it (configs 3 / 5 / 6:
    // depth 22 / 28 / 22).
    static constexpr int kSahDepth = 64;

    // Builds the subtree of the range [b, e) as node `id` (its descendants
    // take ids id + 1 .. id + 2m - 2) at depth `level`; returns its depth
    // below id.
    int build(int id, int b, int e, unsigned threads, int level = 0) {
        BNode& nd = nodes[id];
        const int m = e - b;
        nd.m = m;
        for (int q = 0; q < 3; ++q) {
            nd.lo[q] = INFINITY;
            nd.hi[q] = -INFINITY;
        }
        for (int i = b; i < e; ++i)
            for (int q = 0; q < 3; ++q) {
                nd.lo[q] = std::min(nd.lo[q], prims[ord[0][i]].lo[q]);
                nd.hi[q] = std::max(nd.hi[q], prims[ord[0][i]].hi[q]);
            }
        if (m == 1) {
            nd.prim = ord[0][b];
            nd.cls = prims[nd.prim].cls;
            return 0;
        }
        int baxis = 0, bpos = m / 2;
        float bcost = 0.0f;
        bool found = false;
        if (level >= kSahDepth) {                     // median of the widest centroid extent
            float ext = -1.0f;
            for (int k = 0; k < 3; ++k) {
                const float x = prims[ord[k][e - 1]].c[k] - prims[ord[k][b]].c[k];
                if (x > ext) {
                    ext = x;
                    baxis = k;
                }
            }
            found = true;
        }
        // ties keep the split nearest the middle: equal costs (coincident
        // boxes) must not peel one primitive off per level
        const auto off_mid = [m](int pos) { return pos > m - pos ? 2 * pos - m : m - 2 * pos; };
        for (int k = 0; k < 3 && level < kSahDepth; ++k) {
            const int* o = ord[k].data();
            float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int i = e - 1; i > b; --i) {
                const Prim& p = prims[o[i]];
                for (int q = 0; q < 3; ++q) {
                    lo[q] = std::min(lo[q], p.lo[q]);
                    hi[q] = std::max(hi[q], p.hi[q]);
                }
                rarea[i] = area(lo, hi);
            }
            for (int q = 0; q < 3; ++q) {
                lo[q] = INFINITY;
                hi[q] = -INFINITY;
            }
            for (int i = b; i < e - 1; ++i) {          // left = [b, i], right = [i + 1, e)
                const Prim& p = prims[o[i]];
                for (int q = 0; q < 3; ++q) {
                    lo[q] = std::min(lo[q], p.lo[q]);
                    hi[q] = std::max(hi[q], p.hi[q]);
                }
                const float cost = (float)(i - b + 1) * area(lo, hi) + (float)(e - 1 - i) * rarea[i + 1];
                if (!found || cost < bcost || (cost == bcost && off_mid(i + 1 - b) < off_mid(bpos))) {
                    found = true;
                    baxis = k;
                    bpos = i + 1 - b;
                    bcost = cost;
                }
            }
        }
        nd.axis = baxis;
        const int mid = b + bpos;
        for (int i = b; i < e; ++i) left[ord[baxis][i]] = i < mid ? 1 : 0;
        for (int k = 0; k < 3; ++k) {
            if (k == baxis) continue;
            int* o = ord[k].data();
            int nl = b, nr = mid;
            for (int i = b; i < e; ++i) tmp[left[o[i]] ? nl++ : nr++] = o[i];
            std::copy(tmp.begin() + b, tmp.begin() + e, o + b);
        }
        const int ml = mid - b;
        nd.left = id + 1;
        nd.right = id + 2 * ml;   // id + 1 + (2 ml - 1)
        int dl, dr;
        if (threads > 1 && m > 16384) {
            std::thread th([&] { dl = build(id + 1, b, mid, threads / 2, level + 1); });
            dr = build(id + 2 * ml, mid, e, threads - threads / 2, level + 1);
            th.join();
        } else {
            dl = build(id + 1, b, mid, 1, level + 1);
            dr = build(id + 2 * ml, mid, e, 1, level + 1);
        }
        nd.cls = std::max(nodes[id + 1].cls, nodes[id + 2 * ml].cls);
        return 1 + std::max(dl, dr);
    }
};

uint64_t fnv(const unsigned char* p, size_t n, uint64_t h) {
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

void put_f(uint32_t* w, float f) { std::memcpy(w, &f, 4); }

// ---- format 2: the 4-wide tree (accel_build.h) ----

// The exponent of an axis: the smallest e with decode(255) >= hi (and 255 *
// 2^e a normal float), so every child bound quantises inside [0, 255].
int wide_exponent(float lo, float hi) {
    const double ext = (double)hi - (double)lo;
    int e = ext > 0.0 ? (int)std::ceil(std::log2(ext / 255.0)) : -100;
    if (e < -100) e = -100;
    while (wide_decode(lo, 255, e) < hi) ++e;
    while (e > -100 && wide_decode(lo, 255, e - 1) >= hi) --e;
    return e;
}

// The largest q with decode(q) <= x, and the smallest q with decode(q) >= x:
// a child's box rounded outward on the node's grid (exact in the kernel's
// float arithmetic, so the decoded box holds the child's true box).
int wide_q_down(float origin, int e, float x) {
    int q = (int)std::floor(((double)x - (double)origin) / std::ldexp(1.0, e));
    q = std::max(0, std::min(255, q));
    while (q > 0 && wide_decode(origin, q, e) > x) --q;
    while (q < 255 && wide_decode(origin, q + 1, e) <= x) ++q;
    return q;
}
int wide_q_up(float origin, int e, float x) {
    int q = (int)std::ceil(((double)x - (double)origin) / std::ldexp(1.0, e));
    q = std::max(0, std::min(255, q));
    while (q < 255 && wide_decode(origin, q, e) < x) ++q;
    while (q > 0 && wide_decode(origin, q - 1, e) >= x) --q;
    return q;
}

struct WideEmitter {
    const Builder& B;
    const unsigned char* vb;
    std::vector<uint32_t>& rec;
    size_t next = 0;              // the next free record

    uint32_t* at(size_t i) { return &rec[16 * i]; }

    // The 2-4 binary nodes a wide node of binary node b holds: b's children,
    // the largest-area internal one replaced by its two until there are 4.
    std::vector<int> collapse(int b) const {
        std::vector<int> c = {B.nodes[b].left, B.nodes[b].right};
        while (c.size() < 4) {
            int best = -1;
            float ba = -1.0f;
            for (size_t i = 0; i < c.size(); ++i) {
                const BNode& n = B.nodes[c[i]];
                if (n.prim >= 0) continue;
                const float a = area(n.lo, n.hi);
                if (a > ba) {
                    ba = a;
                    best = (int)i;
                }
            }
            if (best < 0) break;
            const int x = c[best];
            c[best] = B.nodes[x].left;
            c.insert(c.begin() + best + 1, B.nodes[x].right);
        }
        return c;
    }

    // A leaf: what the triangle test reads in the first 48 bytes, the rest of
    // its exact box (read only for a hit that would be taken) in the last 16.
    void leaf(int b, size_t idx) {
        const Prim& p = B.prims[B.nodes[b].prim];
        const BNode& nd = B.nodes[b];
        uint32_t* w = at(idx);
        const unsigned char* v = vb + (size_t)p.tri * 48;
        float x[9];
        for (int j = 0; j < 3; ++j) std::memcpy(&x[3 * j], v + 16 * j, 12);
        const float e1[3] = {x[3] - x[0], x[4] - x[1], x[5] - x[2]};
        const float e2[3] = {x[6] - x[0], x[7] - x[1], x[8] - x[2]};
        w[0] = (uint32_t)p.tri | (1u << 30) | (p.cls >= kAccelClassMin ? 1u << 29 : 0u);
        for (int j = 0; j < 3; ++j) {
            put_f(&w[1 + j], x[j]);
            put_f(&w[4 + j], e1[j]);
            put_f(&w[8 + j], e2[j]);
        }
        put_f(&w[7], nd.lo[0]);
        put_f(&w[11], nd.lo[1]);
        put_f(&w[12], nd.lo[2]);
        put_f(&w[13], nd.hi[0]);
        put_f(&w[14], nd.hi[1]);
        put_f(&w[15], nd.hi[2]);
    }

    // Writes binary node b (internal) as the wide node at idx, its children
    // as one contiguous block of records, and their subtrees after it.
    void node(int b, size_t idx) {
        const BNode& nd = B.nodes[b];
        const std::vector<int> c = collapse(b);
        const size_t base = next;
        next += c.size();
        uint32_t* w = at(idx);
        int e[3];
        for (int q = 0; q < 3; ++q) {
            put_f(&w[q], nd.lo[q]);
            e[q] = wide_exponent(nd.lo[q], nd.hi[q]);
        }
        w[3] = (uint32_t)(uint8_t)(int8_t)e[0] | (uint32_t)(uint8_t)(int8_t)e[1] << 8 |
               (uint32_t)(uint8_t)(int8_t)e[2] << 16 | (uint32_t)c.size() << 24;
        uint32_t flags = 0;
        for (size_t i = 0; i < c.size(); ++i) {
            const BNode& ch = B.nodes[c[i]];
            for (int q = 0; q < 3; ++q) {
                w[4 + q] |= (uint32_t)wide_q_down(nd.lo[q], e[q], ch.lo[q]) << (8 * i);
                w[7 + q] |= (uint32_t)wide_q_up(nd.lo[q], e[q], ch.hi[q]) << (8 * i);
            }
            uint32_t f = 0;
            if (ch.prim >= 0) {
                f |= 1u;                                            // a leaf
                if (ch.cls >= kAccelClassMin) f |= 2u;              // thin: entered whenever hit
            } else if (ch.cls >= kAccelClassMin) {
                f |= 4u;                                            // a subtree with a wider margin
            }
            flags |= f << (8 * i);
        }
        w[10] = (uint32_t)base | (uint32_t)std::min(nd.cls, 31) << 27;
        w[11] = flags;
        for (size_t i = 0; i < c.size(); ++i) {
            if (B.nodes[c[i]].prim >= 0) leaf(c[i], base + i);
            else node(c[i], base + i);
        }
    }
};

void emit_wide(const Builder& B, const unsigned char* vb, AccelHost* out) {
    const size_t m = B.prims.size();
    out->rec.assign(16 * (2 * m + 1), 0u);             // an upper bound; trimmed below
    WideEmitter E{B, vb, out->rec};
    E.next = 1;
    out->root_leaf = B.nodes[0].prim >= 0 ? 1 : 0;
    if (out->root_leaf) E.leaf(0, 0);
    else E.node(0, 0);
    out->slots = (int)E.next;
    out->rec.resize(16 * (E.next + 1));                 // + one record of zero padding
    std::fill(out->rec.end() - 16, out->rec.end(), 0u);
}


}  // namespace

// The float decode the kernel performs: origin + q * 2^e, rounded once.
float wide_decode(float origin, int q, int e) { return origin + (float)q * std::ldexp(1.0f, e); }

int accel_class(const float e1[3], const float e2[3]) {
    const double a[3] = {e1[0], e1[1], e1[2]}, b[3] = {e2[0], e2[1], e2[2]};
    const double c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
    const double s = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]) /
                     (std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]) * std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]));
    if (!(s > 0.0)) return 31;                        // a zero edge or parallel edges (never hit: det = 0)
    const int k = (int)std::floor(-std::log2(s));
    return k < 0 ? 0 : (k > 31 ? 31 : k);
}

float accel_relax(int cls) {
    if (cls < kAccelClassMin) return 1.0f + 1.0f / 1024.0f;
    // 1 + 2^(cls - 16), rounded up to a float (exact for every class in 7..31)
    return 1.0f + std::ldexp(1.0f, cls - 16);
}

uint16_t half_bits_down(float x) {
    if (std::isnan(x)) return 0x7E00u;
    const uint16_t sign = std::signbit(x) ? 0x8000u : 0u;
    if (x == 0.0f) return sign;
    if (std::isinf(x)) return (uint16_t)(sign | 0x7C00u);
    int E;
    (void)std::frexp(x, &E);                          // |x| in [2^(E-1), 2^E)
    const int e = std::max(E - 1, -14);               // the half exponent (subnormals: -14)
    const float ulp = std::ldexp(1.0f, e - 10);
    float r = std::floor(x / ulp) * ulp;              // exact: x / ulp is a power-of-2 scaling
    if (r > 65504.0f) r = 65504.0f;
    if (r < -65504.0f) return 0xFC00u;                // -inf
    if (r == 0.0f) return sign;                       // (only for x >= 0: floor of a negative is < 0)
    const uint16_t rs = std::signbit(r) ? 0x8000u : 0u;
    const float a = std::fabs(r);
    int Ea;
    (void)std::frexp(a, &Ea);
    const int ea = Ea - 1;
    if (ea >= -14)                                    // normal: a = (1 + m / 1024) * 2^ea
        return (uint16_t)(rs | ((ea + 15) << 10) | ((uint32_t)std::ldexp(a, 10 - ea) - 1024u));
    return (uint16_t)(rs | (uint32_t)std::ldexp(a, 24));   // subnormal: a = m * 2^-24
}

int accel_build(const void* vertices, size_t vertex_bytes, const void* materials, size_t material_bytes,
                const void* bvh_nodes, size_t bvh_bytes, int n_layouts, int n_threads, AccelHost* out,
                std::string* err, int format, int64_t cap_slots) {
    *out = AccelHost{};
    if (format < 0 || format > 2) {
        *err = "accel: format must be 0, 1 or 2";
        return -1;
    }
    out->format = format;
    const int W = format == 1 ? 4 : 8;                // words per slot
    const int64_t LS = format == 1 ? 4 : 2;           // slots per leaf
#ifdef ACCEL_TIMING
    const auto t_start = std::chrono::steady_clock::now();
#endif
    if (n_layouts != 1 && n_layouts != 8) {
        *err = "accel: n_layouts must be 1 or 8";
        return -1;
    }
    if (format == 2) n_layouts = 1;                   // the wide walk orders children by t_enter
    out->n_layouts = n_layouts;
    const size_t n_nodes = bvh_bytes / 48, n_tris = vertex_bytes / 48, n_mats = material_bytes / 16;
    const unsigned char* nb = static_cast<const unsigned char*>(bvh_nodes);
    const unsigned char* vb = static_cast<const unsigned char*>(vertices);
    const unsigned char* mb = static_cast<const unsigned char*>(materials);
    if (n_nodes == 0) {           // empty scene: no slots (two of padding), every ray misses
        out->rec.assign(16, 0u);                      // 64 B of padding
        return 0;
    }
    (void)kWideCap;

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
    ACCEL_T("leaves hashed");
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
        {
            const unsigned char* v = vb + (size_t)p.tri * 48;
            float x[9];
            for (int j = 0; j < 3; ++j) std::memcpy(&x[3 * j], v + 16 * j, 12);
            const float e1[3] = {x[3] - x[0], x[4] - x[1], x[5] - x[2]};
            const float e2[3] = {x[6] - x[0], x[7] - x[1], x[8] - x[2]};
            p.cls = accel_class(e1, e2);
        }
        B.prims.push_back(p);
    }
    const int m = (int)B.prims.size();
    out->n_prims = m;
    ACCEL_T("duplicates dropped");
    // a subtree of k triangles: k - 1 internal nodes (1 slot) and k leaves
    const auto span = [LS](int64_t k) { return (LS + 1) * k - 1; };
    // format 2: m leaf records and at most m - 1 wide nodes (64 B each)
    const int64_t slots = format == 2 ? 2 * (int64_t)m - 1 : span(m);
    int64_t cap = format == 1 ? (int64_t)(1u << 30) - 8 : format == 2 ? kWideCap : (int64_t)(1u << 27) - 4;
    if (cap_slots > 0 && cap_slots < cap) cap = cap_slots;
    if (slots * n_layouts + 8 > cap) {
        *err = "accel: " + std::to_string(m) + " triangles: " + std::to_string(n_layouts) + " layouts exceed " +
               std::to_string(cap) + " slots";
        return kAccelTooBig;
    }

    // 2. the tree
    {
        std::vector<std::thread> th;
        for (int k = 0; k < 3; ++k)
            th.emplace_back([&B, m, k] {
                B.ord[k].resize(m);
                for (int i = 0; i < m; ++i) B.ord[k][i] = i;
                std::sort(B.ord[k].begin(), B.ord[k].end(), [&](int x, int y) {
                    return B.prims[x].c[k] != B.prims[y].c[k] ? B.prims[x].c[k] < B.prims[y].c[k] : x < y;
                });
            });
        for (auto& t : th) t.join();
    }
    ACCEL_T("axes sorted");
    B.left.assign(m, 0);
    B.tmp.assign(m, 0);
    B.rarea.assign(m, 0.0f);
    B.nodes.resize(2 * (size_t)m - 1);
    const unsigned hw = n_threads > 0 ? (unsigned)n_threads : std::max(1u, std::thread::hardware_concurrency());
    out->depth = B.build(0, 0, m, std::min(hw, 64u));
    out->max_class = B.nodes[0].cls;
    out->relax_max = accel_relax(B.nodes[0].cls);
    for (const Prim& p : B.prims) out->n_thin += p.cls >= kAccelClassMin ? 1 : 0;
    ACCEL_T("tree built");
    {
        const float a0 = area(B.nodes[0].lo, B.nodes[0].hi);
        double s = 0.0;
        for (const BNode& nd : B.nodes) s += a0 > 0.0f ? (double)area(nd.lo, nd.hi) / a0 : 1.0;
        out->sah = s;
    }

    if (format == 2) {
        emit_wide(B, vb, out);
        ACCEL_T("wide records written");
        return 0;
    }

    // 3. the layouts: preorder, near child first per the layout's sign bits
    out->slots = (int)slots;
    out->root_leaf = B.nodes[0].prim >= 0 ? 1 : 0;
    const size_t total = (size_t)slots * (size_t)n_layouts;
    out->rec.assign((size_t)W * total + 16, 0u);
    std::vector<uint8_t> leaf_at(total + 1, 0);
    auto emit = [&](int o) {
        const size_t base = (size_t)o * (size_t)slots;
        struct Item { int node; size_t pos; };
        std::vector<Item> st;
        st.push_back({0, base});
        while (!st.empty()) {
            const Item it = st.back();
            st.pop_back();
            const BNode& nd = B.nodes[it.node];
            uint32_t* w = &out->rec[(size_t)W * it.pos];
            if (nd.prim >= 0 || format == 0) {
                for (int q = 0; q < 3; ++q) {
                    put_f(&w[q], nd.lo[q]);
                    put_f(&w[4 + q], nd.hi[q]);
                }
            } else {
                w[0] = half_bits_down(nd.lo[0]) | (uint32_t)half_bits_down(nd.lo[1]) << 16;
                w[1] = half_bits_down(nd.lo[2]) | (uint32_t)half_bits_up(nd.hi[0]) << 16;
                w[2] = half_bits_up(nd.hi[1]) | (uint32_t)half_bits_up(nd.hi[2]) << 16;
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
                // | L(next) << 31, below; bit 29: a thin triangle (class >= kAccelClassMin), entered
                // whenever the slab test passes, whatever closest_t
                w[3] = (uint32_t)p.tri | (1u << 30) | (p.cls >= kAccelClassMin ? kAccelForce : 0u);
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
            const size_t skip = it.pos + (size_t)span(nd.m);
            w[3] = (uint32_t)skip;                                 // | L(skip) << 31, below
            if (format == 0 && nd.cls >= kAccelClassMin)           // a thin triangle below: entered whenever
                w[3] |= kAccelForce;                               //   its slab test passes
            const size_t pos2 = it.pos + 1 + (size_t)span(B.nodes[first].m);
            st.push_back({second, pos2});
            st.push_back({first, it.pos + 1});
        }
        // the L bits: an internal node's skip and first child, a leaf's successor
        const size_t end = base + (size_t)slots;
        auto L = [&](size_t s) -> uint32_t { return s < end && leaf_at[s] ? 1u : 0u; };
        for (size_t s = base; s < end;) {
            uint32_t* w = &out->rec[(size_t)W * s];
            if (leaf_at[s]) {
                w[3] |= L(s + (size_t)LS) << 31;
                s += (size_t)LS;
            } else if (format == 0) {
                w[3] |= L(w[3] & ~kAccelForce) << 31;
                w[7] |= L(s + 1) << 31;                   // a sign test in the walk
                s += 1;
            } else {
                w[3] |= L(w[3]) << 31 | L(s + 1) << 30;
                s += 1;
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (int o = 0; o < n_layouts; ++o) th.emplace_back(emit, o);
        for (auto& t : th) t.join();
    }
    ACCEL_T("layouts written");
    return 0;
}

int accel_build_fit(const void* vertices, size_t vertex_bytes, const void* materials, size_t material_bytes,
                    const void* bvh_nodes, size_t bvh_bytes, int n_layouts, AccelHost* out, std::string* err,
                    int format, int64_t cap_slots) {
    int rc = accel_build(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, bvh_bytes, n_layouts, 0, out,
                         err, format, cap_slots);
    if (rc == kAccelTooBig && n_layouts == 8)
        rc = accel_build(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, bvh_bytes, 1, 0, out, err,
                         format, cap_slots);
    return rc;
}

}  // namespace rtamd
