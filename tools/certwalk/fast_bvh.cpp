// fast_bvh.cpp — builder of the certified walk's BVH (fast_bvh.h).
//
// Inputs are the reference's own buffers: 48-B vertex records, three per
// flattened triangle (SceneBuilder.java:95-99), and the 48-B preorder nodes
// (BVHFlattener.java:51-97: leaf data = -(tri+1), count = -1; internal data =
// left = i+1, count = right).
#include "fast_bvh.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

namespace rtamd {
namespace fast {

namespace {

constexpr double kU = 0x1p-24;                     // unit roundoff of binary32
double gam(int k) { return k * kU / (1.0 - k * kU); }

struct RefNode {
    float lo[3], hi[3];
    int32_t data, count;
};

struct Item {
    float lo[3], hi[3];      // box of the real float vertices
    float c[3];              // box centre (SAH key)
};

struct Stats {               // what a child's margin constants depend on
    float lo[3], hi[3];
    double E = 0.0;          // max |e1|_2, |e2|_2
    double A2min = std::numeric_limits<double>::infinity();   // min |e1 x e2|
};

float round_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
}

float round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
}

class Builder {
public:
    Builder(const BuildParams& p, Bvh* out, const std::vector<Item>& items) : p_(p), out_(out), items_(items) {}

    void run(std::vector<int>& idx) {
        idx_ = &idx;
        if (idx.empty()) return;
        out_->nodes.reserve(2 * idx.size());
        out_->tris.clear();
        out_->tris.reserve(tris_in_.size());
        if (idx.size() == 1) {
            // The root is always an internal node: one triangle goes in both
            // children (testing it twice changes nothing: equal t, equal index).
            out_->nodes.emplace_back();
            const int32_t leaf = emit_leaf(0, 1);
            for (int c = 0; c < 2; ++c) {
                out_->nodes[0].child[c] = leaf;
                fill_child(out_->nodes[0].c[c], 0, 1);
            }
            out_->depth = 1;
            return;
        }
        if (p_.orient_classes > 1) {
            build_by_orientation(idx);
            return;
        }
        build(0, (int)idx.size(), 1, true);
    }

    // Orders the caller's triangles to match emitted leaves.
    std::vector<Tri> tris_in_;

private:
    const BuildParams& p_;
    Bvh* out_;
    const std::vector<Item>& items_;
    std::vector<int>* idx_ = nullptr;

    int32_t emit_leaf(int b, int n) {
        const int first = (int)out_->tris.size();
        for (int k = 0; k < n; ++k) out_->tris.push_back(tris_in_[(*idx_)[b + k]]);
        return make_leaf(first, n);
    }

    static double area(const float lo[3], const float hi[3]) {
        const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
        return 2.0 * (x * y + y * z + z * x);
    }

    // Returns the split position (b < m < e), or -1 for a leaf.
    int split(int b, int e, bool force) {
        std::vector<int>& idx = *idx_;
        const int n = e - b;
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int k = b; k < e; ++k) {
            const Item& it = items_[idx[k]];
            for (int a = 0; a < 3; ++a) {
                clo[a] = std::min(clo[a], it.c[a]);
                chi[a] = std::max(chi[a], it.c[a]);
                blo[a] = std::min(blo[a], it.lo[a]);
                bhi[a] = std::max(bhi[a], it.hi[a]);
            }
        }
        const double parea = std::max(area(blo, bhi), 1e-30);
        const int B = std::max(2, p_.bins);
        double best = INFINITY;
        int best_axis = -1, best_bin = -1;
        std::vector<int> cnt(B);
        std::vector<float> lo(3 * B), hi(3 * B);
        std::vector<double> rarea(B);
        std::vector<int> rcnt(B);
        for (int a = 0; a < 3; ++a) {
            const double ext = (double)chi[a] - clo[a];
            if (!(ext > 0.0)) continue;
            std::fill(cnt.begin(), cnt.end(), 0);
            std::fill(lo.begin(), lo.end(), INFINITY);
            std::fill(hi.begin(), hi.end(), -INFINITY);
            const double sc = B / ext;
            for (int k = b; k < e; ++k) {
                const Item& it = items_[idx[k]];
                int bin = std::min(B - 1, (int)((it.c[a] - (double)clo[a]) * sc));
                ++cnt[bin];
                for (int q = 0; q < 3; ++q) {
                    lo[3 * bin + q] = std::min(lo[3 * bin + q], it.lo[q]);
                    hi[3 * bin + q] = std::max(hi[3 * bin + q], it.hi[q]);
                }
            }
            float rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY};
            int rc = 0;
            for (int bin = B - 1; bin > 0; --bin) {
                rc += cnt[bin];
                for (int q = 0; q < 3; ++q) {
                    rl[q] = std::min(rl[q], lo[3 * bin + q]);
                    rh[q] = std::max(rh[q], hi[3 * bin + q]);
                }
                rcnt[bin] = rc;
                rarea[bin] = rc ? area(rl, rh) : 0.0;
            }
            float ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
            int lc = 0;
            for (int bin = 0; bin < B - 1; ++bin) {
                lc += cnt[bin];
                for (int q = 0; q < 3; ++q) {
                    ll[q] = std::min(ll[q], lo[3 * bin + q]);
                    lh[q] = std::max(lh[q], hi[3 * bin + q]);
                }
                if (lc == 0 || rcnt[bin + 1] == 0) continue;
                const double c = (lc * area(ll, lh) + rcnt[bin + 1] * rarea[bin + 1]) / parea;
                if (c < best) {
                    best = c;
                    best_axis = a;
                    best_bin = bin;
                }
            }
        }
        // Costs in units of one triangle test; a node step costs about one.
        const double leaf_cost = n;
        const double split_cost = 1.0 + best;
        if (!force && n <= p_.leaf_max && leaf_cost <= split_cost) return -1;
        if (best_axis < 0) {
            // all centres coincide: split by count
            if (!force && n <= p_.leaf_max) return -1;
            return b + n / 2;
        }
        const double ext = (double)chi[best_axis] - clo[best_axis];
        const double sc = B / ext;
        auto mid = std::partition(idx.begin() + b, idx.begin() + e, [&](int i) {
            const int bin = std::min(B - 1, (int)((items_[i].c[best_axis] - (double)clo[best_axis]) * sc));
            return bin <= best_bin;
        });
        int m = (int)(mid - idx.begin());
        if (m <= b || m >= e) m = b + n / 2;
        return m;
    }

    // Experimental: the top levels split the triangles by the direction class
    // of their normal line, so every class subtree has a narrow normal cone.
    void build_by_orientation(std::vector<int>& idx) {
        static const double dirs[13][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {1, 1, 0}, {1, -1, 0}, {1, 0, 1}, {1, 0, -1},
                                           {0, 1, 1}, {0, 1, -1}, {1, 1, 1}, {1, 1, -1}, {1, -1, 1}, {-1, 1, 1}};
        const int K = p_.orient_classes >= 13 ? 13 : 3;
        std::vector<int> cls(tris_in_.size(), 0);
        for (size_t i = 0; i < tris_in_.size(); ++i) {
            const Tri& T = tris_in_[i];
            const double cx = (double)T.e1[1] * T.e2[2] - (double)T.e1[2] * T.e2[1];
            const double cy = (double)T.e1[2] * T.e2[0] - (double)T.e1[0] * T.e2[2];
            const double cz = (double)T.e1[0] * T.e2[1] - (double)T.e1[1] * T.e2[0];
            double best = -1.0;
            for (int k = 0; k < K; ++k) {
                const double l = std::sqrt(dirs[k][0] * dirs[k][0] + dirs[k][1] * dirs[k][1] + dirs[k][2] * dirs[k][2]);
                const double v = std::fabs(cx * dirs[k][0] + cy * dirs[k][1] + cz * dirs[k][2]) / l;
                if (v > best) { best = v; cls[i] = k; }
            }
        }
        std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return cls[a] < cls[b]; });
        std::vector<std::pair<int, int>> ranges;
        for (size_t k = 0; k < idx.size();) {
            size_t e = k;
            while (e < idx.size() && cls[idx[e]] == cls[idx[k]]) ++e;
            ranges.push_back({(int)k, (int)e});
            k = e;
        }
        if (ranges.size() == 1) {
            build(0, (int)idx.size(), 1, true);
            return;
        }
        build_group(ranges, 0, (int)ranges.size(), 1);
    }

    int32_t build_group(const std::vector<std::pair<int, int>>& g, int gb, int ge, int depth) {
        if (ge - gb == 1) return build(g[gb].first, g[gb].second, depth, g[gb].second - g[gb].first > 1);
        const int gm = (gb + ge) / 2;
        const int self = (int)out_->nodes.size();
        out_->nodes.emplace_back();
        const int32_t l = build_group(g, gb, gm, depth + 1);
        const int32_t r = build_group(g, gm, ge, depth + 1);
        Node& nd = out_->nodes[self];
        nd.child[0] = l;
        nd.child[1] = r;
        fill_child(nd.c[0], g[gb].first, g[gm - 1].second);
        fill_child(nd.c[1], g[gm].first, g[ge - 1].second);
        out_->depth = std::max(out_->depth, depth);
        return self;
    }

    // Builds the subtree of idx[b, e) as node `self` (already allocated when
    // called for a child) and returns the child reference.
    int32_t build(int b, int e, int depth, bool root) {
        const int n = e - b;
        out_->depth = std::max(out_->depth, depth);
        const int m = split(b, e, root || n > p_.leaf_max);
        if (m < 0) return emit_leaf(b, n);
        const int self = (int)out_->nodes.size();
        out_->nodes.emplace_back();
        const int32_t l = build(b, m, depth + 1, false);
        const int32_t r = build(m, e, depth + 1, false);
        Node& nd = out_->nodes[self];
        nd.child[0] = l;
        nd.child[1] = r;
        fill_child(nd.c[0], b, m);
        fill_child(nd.c[1], m, e);
        return self;
    }

    void fill_child(ChildBox& cb, int b, int e) {
        const std::vector<int>& idx = *idx_;
        Stats st;
        for (int a = 0; a < 3; ++a) {
            st.lo[a] = INFINITY;
            st.hi[a] = -INFINITY;
        }
        // normals of the Möller–Trumbore triangles (v0, v0+e1, v0+e2), in double
        std::vector<double> nv;
        nv.reserve(3 * (size_t)(e - b));
        double ref[3] = {0, 0, 0}, ref_a2 = -1.0;
        for (int k = b; k < e; ++k) {
            const Item& it = items_[idx[k]];
            const Tri& T = tris_in_[idx[k]];
            for (int a = 0; a < 3; ++a) {
                st.lo[a] = std::min(st.lo[a], it.lo[a]);
                st.hi[a] = std::max(st.hi[a], it.hi[a]);
            }
            const double ax = T.e1[0], ay = T.e1[1], az = T.e1[2];
            const double bx = T.e2[0], by = T.e2[1], bz = T.e2[2];
            st.E = std::max(st.E, std::sqrt(ax * ax + ay * ay + az * az) * (1.0 + 1e-15));
            st.E = std::max(st.E, std::sqrt(bx * bx + by * by + bz * bz) * (1.0 + 1e-15));
            const double cx = ay * bz - az * by, cy = az * bx - ax * bz, cz = ax * by - ay * bx;
            const double a2 = std::sqrt(cx * cx + cy * cy + cz * cz);
            st.A2min = std::min(st.A2min, a2 * (1.0 - 1e-12));
            if (a2 > 0.0) {
                nv.push_back(cx / a2);
                nv.push_back(cy / a2);
                nv.push_back(cz / a2);
                if (a2 > ref_a2) {
                    ref_a2 = a2;
                    ref[0] = cx / a2;
                    ref[1] = cy / a2;
                    ref[2] = cz / a2;
                }
            }
        }
        for (int a = 0; a < 3; ++a) {
            cb.lo[a] = st.lo[a];
            cb.hi[a] = st.hi[a];
        }
        // Cone of normal lines: orient each normal towards ref, average, then
        // the widest line angle from the (float-rounded) axis.
        double s[3] = {0, 0, 0};
        for (size_t k = 0; k < nv.size(); k += 3) {
            const double dd = nv[k] * ref[0] + nv[k + 1] * ref[1] + nv[k + 2] * ref[2];
            const double sg = dd < 0.0 ? -1.0 : 1.0;
            s[0] += sg * nv[k];
            s[1] += sg * nv[k + 1];
            s[2] += sg * nv[k + 2];
        }
        const double sl = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
        float af[3] = {0.f, 0.f, 1.f};
        if (sl > 0.0)
            for (int a = 0; a < 3; ++a) af[a] = (float)(s[a] / sl);
        const double al = std::sqrt((double)af[0] * af[0] + (double)af[1] * af[1] + (double)af[2] * af[2]);
        double cmin = 1.0;   // min |cos| between the axis line and a normal line
        for (size_t k = 0; k < nv.size(); k += 3) {
            const double c = std::fabs(af[0] * nv[k] + af[1] * nv[k + 1] + af[2] * nv[k + 2]) / al;
            cmin = std::min(cmin, c);
        }
        const double alpha = std::min(0.5 * M_PI, std::acos(std::min(1.0, cmin)) + 1e-7);
        for (int a = 0; a < 3; ++a) cb.axis[a] = af[a];
        if (nv.empty()) {
            cb.ca = 0.0f;   // no normal: no cone bound (|det| floor only)
            cb.sa = 1.0f;
        } else {
            cb.ca = round_down(std::cos(alpha));
            cb.sa = round_up(std::sin(alpha));
        }
        cb.a2min = std::isfinite(st.A2min) ? round_down(st.A2min) : 0.0f;
        cb.emax = round_up(st.E);
    }
};

}  // namespace

int build_fast_bvh(const void* vertices, size_t vertex_bytes, const void* bvh_nodes, size_t bvh_bytes,
                   const BuildParams& p, Bvh* out, std::string* err) {
    *out = Bvh();
    if (vertex_bytes % 48 || bvh_bytes % 48) {
        if (err) *err = "buffer sizes are not multiples of 48 bytes";
        return -1;
    }
    if (p.leaf_max < 1 || p.leaf_max > kLeafMaxLimit) {
        if (err) *err = "leaf_max out of range";
        return -1;
    }
    const size_t n_tris = vertex_bytes / 48, n_nodes = bvh_bytes / 48;
    const unsigned char* nb = (const unsigned char*)bvh_nodes;
    const float* vf = (const float*)vertices;
    std::vector<RefNode> rn(n_nodes);
    for (size_t i = 0; i < n_nodes; ++i) {
        memcpy(rn[i].lo, nb + 48 * i, 12);
        memcpy(rn[i].hi, nb + 48 * i + 16, 12);
        memcpy(&rn[i].data, nb + 48 * i + 32, 4);
        memcpy(&rn[i].count, nb + 48 * i + 36, 4);
    }
    // Certificate preconditions: strictly positive boxes,
    // children nested in parents, left child = i + 1.
    out->certifiable = true;
    for (size_t i = 0; i < n_nodes && out->certifiable; ++i) {
        const RefNode& r = rn[i];
        for (int a = 0; a < 3; ++a)
            if (!(r.lo[a] < r.hi[a])) {
                out->certifiable = false;
                out->why_not = "node " + std::to_string(i) + " has a box of zero or negative extent";
            }
        if (r.count >= 0) {
            const int32_t ch[2] = {r.data, r.count};
            if (r.data != (int32_t)i + 1) {
                out->certifiable = false;
                out->why_not = "node " + std::to_string(i) + " is not in the reference's preorder";
            }
            for (int c = 0; c < 2; ++c) {
                if (ch[c] < 0 || (size_t)ch[c] >= n_nodes) {
                    if (err) *err = "child index out of range";
                    return -1;
                }
                const RefNode& k = rn[ch[c]];
                for (int a = 0; a < 3; ++a)
                    if (!(r.lo[a] <= k.lo[a] && k.hi[a] <= r.hi[a])) {
                        out->certifiable = false;
                        out->why_not = "node " + std::to_string(ch[c]) + " is not inside its parent";
                    }
            }
        }
    }
    // Leaves, in preorder; a sibling leaf with the same triangle and box as the
    // left one (BVHBuilder.java:60-62 duplicates a lone triangle) is dropped:
    // it can only tie with the left leaf, which wins ties.
    std::vector<Tri> tris;
    std::vector<Item> items;
    std::vector<char> dup(n_nodes, 0);
    for (size_t i = 0; i < n_nodes; ++i) {
        const RefNode& r = rn[i];
        if (r.count >= 0) {
            const RefNode& L = rn[r.data];
            const RefNode& R = rn[r.count];
            if (L.count < 0 && R.count < 0) {
                const int kl = -(L.data + 1), kr = -(R.data + 1);
                if (kl >= 0 && kr >= 0 && (size_t)kl < n_tris && (size_t)kr < n_tris &&
                    memcmp(vf + 12 * (size_t)kl, vf + 12 * (size_t)kr, 48) == 0 && memcmp(L.lo, R.lo, 12) == 0 &&
                    memcmp(L.hi, R.hi, 12) == 0)
                    dup[r.count] = 1;
            }
            continue;
        }
        out->n_ref_leaves++;
        if (dup[i]) continue;
        const int k = -(r.data + 1);
        if (k < 0 || (size_t)k >= n_tris) {
            if (err) *err = "leaf triangle index out of range";
            return -1;
        }
        const float* v = vf + 12 * (size_t)k;
        Tri t;
        Item it;
        for (int a = 0; a < 3; ++a) {
            t.v0[a] = v[a];
            t.e1[a] = v[4 + a] - v[a];
            t.e2[a] = v[8 + a] - v[a];
            it.lo[a] = std::min(std::min(v[a], v[4 + a]), v[8 + a]);
            it.hi[a] = std::max(std::max(v[a], v[4 + a]), v[8 + a]);
            it.c[a] = 0.5f * (it.lo[a] + it.hi[a]);
            out->lscene = std::max(out->lscene, std::max(std::fabs(it.lo[a]), std::fabs(it.hi[a])));
        }
        t.tri = k;
        t.leaf = (int32_t)i;
        tris.push_back(t);
        items.push_back(it);
    }
    for (int a = 0; a < 3; ++a) {
        out->root_lo[a] = INFINITY;
        out->root_hi[a] = -INFINITY;
    }
    for (const Item& it : items)
        for (int a = 0; a < 3; ++a) {
            out->root_lo[a] = std::min(out->root_lo[a], it.lo[a]);
            out->root_hi[a] = std::max(out->root_hi[a], it.hi[a]);
        }
    if (items.empty())
        for (int a = 0; a < 3; ++a) out->root_lo[a] = out->root_hi[a] = 0.f;
    std::vector<int> idx(items.size());
    for (size_t k = 0; k < idx.size(); ++k) idx[k] = (int)k;
    Builder b(p, out, items);
    out->mc.kdet = 4.2150e-7f;
    out->mc.g2 = 1.19210e-7f * 1.0001f;
    out->mc.g3 = 1.78814e-7f * 1.0001f;
    out->mc.ulscene = round_up(1.01 * kU * out->lscene);
    b.tris_in_ = std::move(tris);
    b.run(idx);
    return 0;
}

}  // namespace fast
}  // namespace rtamd
