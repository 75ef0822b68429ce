// fastpath_sim.cpp — analysis aid (not product): compares, segment by
// segment on real paths of a BASELINE config, the reference's preorder walk
// with a front-to-back walk over a separate SAH BVH whose culling carries
// rigorous Möller–Trumbore error margins, followed by the one-box check that
// proves the result equals the reference's.  Reports work
// per segment, the per-wave lockstep cost, fallbacks and any mismatch.
//
//   g++ -O2 -std=c++17 -ffp-contract=off -fopenmp tools/fastpath_sim.cpp -o /tmp/fastpath_sim
//   /tmp/fastpath_sim DIR [row_step] [leaf_max] [sinb] [per_node_S]
// DIR holds verts.bin / nodes.bin / mats.bin / cam.bin / meta.txt (tools/dump_config.py).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <string>

#include "fast_bvh.h"
#include "fast_margin.h"

using namespace rtamd::fast;

namespace {

struct V3 { float x, y, z; };
static V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
static V3 scl(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static V3 crs(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static V3 nrm(V3 a) { float l = std::sqrt(dot(a, a)); return {a.x / l, a.y / l, a.z / l}; }

static uint32_t pcg(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
static float rnd(uint32_t& s) { s = pcg(s); return (float)s / 4294967296.0f; }
static V3 in_sphere(uint32_t& s) {
    s = pcg(pcg(pcg(s)));
    for (int it = 0; it < 65536; ++it) {
        float a = rnd(s), b = rnd(s), c = rnd(s);
        V3 p = {a * 2.f - 1.f, b * 2.f - 1.f, c * 2.f - 1.f};
        if (dot(p, p) < 1.f) return p;
    }
    return {0, 0, 0};
}

static std::vector<char> slurp(const std::string& p) {
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) { perror(p.c_str()); exit(1); }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<char> b(n);
    if (fread(b.data(), 1, n, f) != (size_t)n) exit(1);
    fclose(f);
    return b;
}

struct RefScene {
    const float* verts;   // 12 floats per triangle
    const float* mats;    // 4 per triangle
    const unsigned char* nodes;
    int n_nodes;
};

static void slab(const float* lo, const float* hi, V3 o, V3 inv, float& te, float& tx) {
    float t0x = (lo[0] - o.x) * inv.x, t1x = (hi[0] - o.x) * inv.x;
    float t0y = (lo[1] - o.y) * inv.y, t1y = (hi[1] - o.y) * inv.y;
    float t0z = (lo[2] - o.z) * inv.z, t1z = (hi[2] - o.z) * inv.z;
    te = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    tx = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
}

static bool tri_test(V3 v0, V3 e1, V3 e2, V3 o, V3 d, float& t) {
    V3 pv = crs(d, e2);
    float det = dot(e1, pv);
    if (det > -0.00001f && det < 0.00001f) return false;
    float id = 1.0f / det;
    V3 s = sub(o, v0);
    float u = id * dot(s, pv);
    if (u < 0.f || u > 1.f) return false;
    V3 q = crs(s, e1);
    float v = id * dot(d, q);
    if (v < 0.f || (u + v) > 1.f) return false;
    t = id * dot(e2, q);
    return t > 0.001f;
}

struct Hit { float t; int tri; int leaf; long visits, tris; };
static long g_extra[4][64];
static bool g_verbose = false;
static thread_local long g_margin_evals = 0;   // [kind][depth]: 0 = kept only by margin (cone), 1 = by margin (det floor), 2 = unbounded, 3 = kept plainly
static std::vector<int> g_depth;

// The reference DFS (compute_dynamic_ray.comp:185-210).
static Hit ref_walk(const RefScene& S, V3 o, V3 d) {
    Hit h{10000.f, -1, -1, 0, 0};
    V3 inv = {1.f / d.x, 1.f / d.y, 1.f / d.z};
    int stk[64], sp = 0;
    stk[sp++] = 0;
    while (sp) {
        int i = stk[--sp];
        const unsigned char* nd = S.nodes + (size_t)i * 48;
        const float* lo = (const float*)nd;
        const float* hi = (const float*)(nd + 16);
        int32_t data, count;
        memcpy(&data, nd + 32, 4);
        memcpy(&count, nd + 36, 4);
        h.visits++;
        float te, tx;
        slab(lo, hi, o, inv, te, tx);
        if (tx > te && tx > 0.001f && te < h.t) {
            if (count < 0) {
                int k = -(data + 1);
                const float* v = S.verts + 12 * (size_t)k;
                V3 v0 = {v[0], v[1], v[2]}, v1 = {v[4], v[5], v[6]}, v2 = {v[8], v[9], v[10]};
                h.tris++;
                float t;
                if (tri_test(v0, sub(v1, v0), sub(v2, v0), o, d, t) && t < h.t) {
                    h.t = t;
                    h.tri = k;
                    h.leaf = i;
                }
            } else {
                stk[sp++] = count;
                stk[sp++] = data;
            }
        }
    }
    return h;
}

struct Stats {
    long seg = 0, ref_visits = 0, ref_tris = 0, f_nodes = 0, f_tris = 0, fallback = 0, mismatch = 0, miss_both = 0;
    long fb_reason[3] = {0, 0, 0};
};

// Front-to-back walk over the fast BVH (mirrors the planned GPU kernel).
static Hit fast_walk(const Bvh& B, V3 o, V3 d, float Sray, bool per_node_S, bool zero_margin, long& nodes,
                     long& tris) {
    Hit h{10000.f, -1, -1, 0, 0};
    V3 inv = {1.f / d.x, 1.f / d.y, 1.f / d.z};
    struct E { int node; float key; };
    E stk[128];
    int sp = 0;
    int cur = 0;   // root node
    if (B.nodes.empty()) return h;
    for (;;) {
        if (cur >= 0) {
            const Node& n = B.nodes[cur];
            ++nodes;
            float key[2];
            bool keep[2];
            for (int c = 0; c < 2; ++c) {
                const ChildBox& cb = n.c[c];
                float r = INFINITY, m = INFINITY;
                const bool bounded = child_margins(cb.lo[0], cb.lo[1], cb.lo[2], cb.hi[0], cb.hi[1], cb.hi[2],
                                                   cb.axis[0], cb.axis[1], cb.axis[2], cb.ca, cb.sa, cb.a2min,
                                                   cb.emax, o.x, o.y, o.z, d.x, d.y, d.z, B.mc.ulscene, r, m);
                if (zero_margin) { r = 1e-4f; m = 0.f; }
                {
                    float tep, txp;
                    slab(cb.lo, cb.hi, o, inv, tep, txp);
                    if (!(txp > tep && txp > 0.001f && tep <= h.t)) ++g_margin_evals;
                }
                (void)Sray; (void)per_node_S;
                const int dep = std::min(63, g_depth[cur]);
                if (!bounded && !zero_margin) { keep[c] = true; key[c] = -INFINITY; __atomic_add_fetch(&g_extra[2][dep], 1, __ATOMIC_RELAXED); continue; }
                {
                    float te0, tx0;
                    slab(cb.lo, cb.hi, o, inv, te0, tx0);
                    const bool plain = tx0 > te0 && tx0 > 0.001f && te0 <= h.t;
                    const float ddot = fabsf(d.x * cb.axis[0] + d.y * cb.axis[1] + d.z * cb.axis[2]);
                    const float sd = sqrtf(fmaxf(0.f, 1.f - ddot * ddot));
                    const bool floor_ = cb.a2min * (ddot * cb.ca - sd * cb.sa) <= 1e-5f;
                    float lo2[3] = {cb.lo[0] - r, cb.lo[1] - r, cb.lo[2] - r}, hi2[3] = {cb.hi[0] + r, cb.hi[1] + r, cb.hi[2] + r};
                    float te1, tx1;
                    slab(lo2, hi2, o, inv, te1, tx1);
                    const bool infl = tx1 > te1 && tx1 > 0.001f && te1 - m <= h.t * (1.0f + 2.4e-7f);
                    if (g_verbose) {
                        const float sd2 = sqrtf(fmaxf(0.f, 1.f - ddot * ddot));
                        fprintf(stderr, "  node %d d%d c%d plain %d infl %d r %.3g m %.3g cb %.3f a2 %.3g emax %.3g size %.3f te0 %.4g tx0 %.4g c %.5g\n", cur, dep, c, plain, infl, r, m, ddot * cb.ca - sd2 * cb.sa, cb.a2min, cb.emax, fmaxf(cb.hi[0]-cb.lo[0], fmaxf(cb.hi[1]-cb.lo[1], cb.hi[2]-cb.lo[2])), te0, tx0, h.t);
                    }
                    if (plain) __atomic_add_fetch(&g_extra[3][dep], 1, __ATOMIC_RELAXED);
                    else if (infl) {
                        __atomic_add_fetch(&g_extra[floor_ ? 1 : 0][dep], 1, __ATOMIC_RELAXED);
                        static int shown = 0;
                        if (floor_ && dep >= 13 && shown < 25) {
                            ++shown;
                            fprintf(stderr, "floor d%d ddot %.4f ca %.4f sa %.4f a2 %.3g emax %.3g r %.3g m %.3g box %.3f..%.3f  te0 %.4g tx0 %.4g c %.4g o %.2f %.2f %.2f\n", dep, ddot, cb.ca, cb.sa, cb.a2min, cb.emax, r, m, cb.lo[1], cb.hi[1], te0, tx0, h.t, o.x, o.y, o.z);
                        }
                    }
                }
                const float lo[3] = {cb.lo[0] - r, cb.lo[1] - r, cb.lo[2] - r};
                const float hi[3] = {cb.hi[0] + r, cb.hi[1] + r, cb.hi[2] + r};
                float te, tx;
                slab(lo, hi, o, inv, te, tx);
                const bool ind = tx > te && tx > 0.001f;
                key[c] = te - m;
                keep[c] = ind && key[c] <= h.t * (1.0f + 2.4e-7f);
            }
            int first = -1, second = -1;
            if (keep[0] && keep[1]) {
                first = key[0] <= key[1] ? 0 : 1;
                second = 1 - first;
            } else if (keep[0]) first = 0;
            else if (keep[1]) first = 1;
            if (second >= 0) stk[sp++] = {n.child[second], key[second]};
            if (first >= 0) {
                int ch = n.child[first];
                if (ch >= 0) { cur = ch; continue; }
                stk[sp++] = {ch, key[first]};   // leaf: tested on pop
            }
            cur = -1;
            continue;
        }
        // pop
        bool got = false;
        while (sp) {
            E e = stk[--sp];
            if (!(e.key <= h.t * (1.0f + 2.4e-7f))) continue;
            if (e.node >= 0) { cur = e.node; got = true; break; }
            // leaf range
            const int first = leaf_first(e.node), cnt = leaf_count(e.node);
            for (int k = 0; k < cnt; ++k) {
                const Tri& T = B.tris[first + k];
                ++tris;
                float t;
                V3 v0 = {T.v0[0], T.v0[1], T.v0[2]}, e1 = {T.e1[0], T.e1[1], T.e1[2]}, e2 = {T.e2[0], T.e2[1], T.e2[2]};
                if (tri_test(v0, e1, e2, o, d, t)) {
                    if (t < h.t || (t == h.t && h.leaf >= 0 && T.leaf < h.leaf)) {
                        h.t = t;
                        h.tri = T.tri;
                        h.leaf = T.leaf;
                    }
                }
            }
        }
        if (!got) break;
    }
    return h;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s DIR [row_step] [leaf_max] [sinb] [per_node_S] [zero]\n", argv[0]); return 2; }
    std::string dir = argv[1];
    int row_step = argc > 2 ? atoi(argv[2]) : 4;
    int leaf_max = argc > 3 ? atoi(argv[3]) : 1;
    bool per_node_S = true;
    bool zero = argc > 4 ? atoi(argv[4]) != 0 : false;
    auto vb = slurp(dir + "/verts.bin"), mb = slurp(dir + "/mats.bin"), nb = slurp(dir + "/nodes.bin"),
         cb = slurp(dir + "/cam.bin");
    int W, H, MB;
    FILE* f = fopen((dir + "/meta.txt").c_str(), "r");
    if (fscanf(f, "%d %d %d", &W, &H, &MB) != 3) return 1;
    fclose(f);
    RefScene S{(const float*)vb.data(), (const float*)mb.data(), (const unsigned char*)nb.data(),
               (int)(nb.size() / 48)};
    const float* cam = (const float*)cb.data();

    Bvh B;
    BuildParams bp;
    bp.leaf_max = leaf_max;
    bp.orient_classes = argc > 5 ? atoi(argv[5]) : 0;
    std::string err;
    if (build_fast_bvh(vb.data(), vb.size(), nb.data(), nb.size(), bp, &B, &err) != 0) {
        fprintf(stderr, "build failed: %s\n", err.c_str());
        return 1;
    }
    fprintf(stderr, "fast bvh: %zu nodes, %zu tris (dedup from %d leaves), depth %d\n", B.nodes.size(),
            B.tris.size(), B.n_ref_leaves, B.depth);
    g_depth.assign(B.nodes.size(), 0);
    for (size_t i = 0; i < B.nodes.size(); ++i)
        for (int c = 0; c < 2; ++c) if (B.nodes[i].child[c] >= 0) g_depth[B.nodes[i].child[c]] = g_depth[i] + 1;
    const float* rb = B.root_lo;
    const float* rh = B.root_hi;

    if (getenv("TRACE_PX")) {
        int px, py;
        sscanf(getenv("TRACE_PX"), "%d,%d", &px, &py);
        g_verbose = true;
        uint32_t seed = (uint32_t)(py * W + px);
        float uu = ((float)px + rnd(seed)) / (float)W;
        float vv = ((float)(H - 1 - py) + rnd(seed)) / (float)H;
        V3 o = {cam[0], cam[1], cam[2]};
        V3 llc = {cam[4], cam[5], cam[6]}, hor = {cam[8], cam[9], cam[10]}, ver = {cam[12], cam[13], cam[14]};
        V3 d = nrm(sub(add(add(llc, scl(hor, uu)), scl(ver, vv)), o));
        g_depth.assign(B.nodes.size(), 0);
        for (size_t i = 0; i < B.nodes.size(); ++i)
            for (int c = 0; c < 2; ++c) if (B.nodes[i].child[c] >= 0) g_depth[B.nodes[i].child[c]] = g_depth[i] + 1;
        long fn = 0, ft = 0;
        Hit q = fast_walk(B, o, d, 0.f, true, false, fn, ft);
        Hit r = ref_walk(S, o, d);
        fprintf(stderr, "fast nodes %ld tris %ld hit %d t %.6g | ref visits %ld hit %d t %.6g\n", fn, ft, q.tri, q.t, r.visits, r.tri, r.t);
        return 0;
    }
    const int rows = (H + row_step - 1) / row_step;
    // per pixel per bounce: iterations (ref, fast)
    std::vector<int32_t> it_ref((size_t)rows * W * MB, 0), it_fast((size_t)rows * W * MB, 0);
    std::vector<int32_t> alu_ref((size_t)rows * W * MB, 0), alu_fast((size_t)rows * W * MB, 0);
    Stats tot;
#pragma omp parallel
    {
        Stats st;
#pragma omp for schedule(dynamic, 1)
        for (int rr = 0; rr < rows; ++rr) {
            const int y = rr * row_step;
            for (int x = 0; x < W; ++x) {
                uint32_t seed = (uint32_t)(y * W + x);
                float uu = ((float)x + rnd(seed)) / (float)W;
                float vv = ((float)(H - 1 - y) + rnd(seed)) / (float)H;
                V3 o = {cam[0], cam[1], cam[2]};
                V3 llc = {cam[4], cam[5], cam[6]}, hor = {cam[8], cam[9], cam[10]}, ver = {cam[12], cam[13], cam[14]};
                V3 d = nrm(sub(add(add(llc, scl(hor, uu)), scl(ver, vv)), o));
                for (int b = 0; b < MB; ++b) {
                    st.seg++;
                    Hit r = ref_walk(S, o, d);
                    st.ref_visits += r.visits;
                    if (r.visits > 600) {
#pragma omp critical
                        fprintf(stderr, "HEAVY px %d,%d b %d visits %ld tris %ld hit %d t %.3f o %.3f %.3f %.3f d %.4f %.4f %.4f\n", x, y, b, r.visits, r.tris, r.tri, r.t, o.x, o.y, o.z, d.x, d.y, d.z);
                    }
                    st.ref_tris += r.tris;
                    float Sray = 0.f;
                    Sray = fmaxf(Sray, fmaxf(fabsf(rb[0] - o.x), fabsf(rh[0] - o.x)));
                    Sray = fmaxf(Sray, fmaxf(fabsf(rb[1] - o.y), fabsf(rh[1] - o.y)));
                    Sray = fmaxf(Sray, fmaxf(fabsf(rb[2] - o.z), fabsf(rh[2] - o.z)));
                    Sray *= 1.0001f;
                    long fn = 0, ft = 0;
                    g_margin_evals = 0;
                    Hit q = fast_walk(B, o, d, Sray, per_node_S, zero, fn, ft);
                    long falu = fn * 56 + g_margin_evals * 60 + ft * 45 + 25;
                    st.f_nodes += fn;
                    st.f_tris += ft;
                    long fast_iters = fn + ft;
                    // verification: the candidate's reference leaf box
                    bool ok = true;
                    if (q.leaf >= 0) {
                        const unsigned char* nd = S.nodes + (size_t)q.leaf * 48;
                        V3 inv = {1.f / d.x, 1.f / d.y, 1.f / d.z};
                        float te, tx;
                        slab((const float*)nd, (const float*)(nd + 16), o, inv, te, tx);
                        bool ind = tx > te && tx > 0.001f;
                        if (!ind) { ok = false; st.fb_reason[0]++; }
                        else if (!(te <= q.t)) { ok = false; st.fb_reason[1]++; }
                        fast_iters += 1;
                    }
                    if (!ok) {
                        st.fallback++;
                        fast_iters += r.visits + r.tris;
                        falu += r.visits * 28 + r.tris * 45;
                    } else {
                        bool same = (q.tri == r.tri) && (q.tri < 0 || memcmp(&q.t, &r.t, 4) == 0);
                        if (!same) {
                            st.mismatch++;
                            if (st.mismatch < 5)
                                fprintf(stderr, "MISMATCH px %d,%d b %d: ref (%d, %.9g) fast (%d, %.9g)\n", x, y, b, r.tri,
                                        r.t, q.tri, q.t);
                        }
                    }
                    const size_t ix = ((size_t)rr * W + x) * MB + b;
                    it_ref[ix] = (int32_t)(r.visits + r.tris);
                    it_fast[ix] = (int32_t)fast_iters;
                    alu_ref[ix] = (int32_t)(r.visits * 28 + r.tris * 45);
                    alu_fast[ix] = (int32_t)falu;
                    // continue the reference path
                    if (r.tri < 0) break;
                    const float* m = S.mats + 4 * (size_t)r.tri;
                    const float* v = S.verts + 12 * (size_t)r.tri;
                    V3 v0 = {v[0], v[1], v[2]}, v1 = {v[4], v[5], v[6]}, v2 = {v[8], v[9], v[10]};
                    V3 n = nrm(crs(sub(v1, v0), sub(v2, v0)));
                    if (dot(d, n) > 0.f) n = scl(n, -1.f);
                    V3 hp = add(o, scl(d, r.t));
                    V3 nd;
                    if (m[3] == 0.f) {
                        V3 ru = nrm(in_sphere(seed));
                        V3 sd = add(n, ru);
                        if (std::sqrt(dot(sd, sd)) < 0.0001f) sd = n;
                        nd = nrm(sd);
                    } else if (m[3] == 1.f || m[3] == 2.f) {
                        float fz = m[3] == 2.f ? 0.3f : 0.f;
                        V3 di = nrm(d);
                        float k = 2.f * dot(n, di);
                        V3 rf = sub(di, scl(n, k));
                        V3 p = in_sphere(seed);
                        nd = nrm(add(rf, scl(p, fz)));
                        if (!(dot(nd, n) > 0.f)) break;
                    } else break;
                    o = hp;
                    d = nd;
                }
            }
        }
#pragma omp critical
        {
            tot.seg += st.seg; tot.ref_visits += st.ref_visits; tot.ref_tris += st.ref_tris;
            tot.f_nodes += st.f_nodes; tot.f_tris += st.f_tris; tot.fallback += st.fallback;
            tot.mismatch += st.mismatch;
            for (int k = 0; k < 3; ++k) tot.fb_reason[k] += st.fb_reason[k];
        }
    }
    printf("segments %ld\n", tot.seg);
    printf("ref : visits/seg %.2f tris/seg %.3f\n", (double)tot.ref_visits / tot.seg, (double)tot.ref_tris / tot.seg);
    printf("fast: nodes/seg %.2f tris/seg %.3f  fallback %ld (ind %ld, te>t %ld)  MISMATCH %ld\n",
           (double)tot.f_nodes / tot.seg, (double)tot.f_tris / tot.seg, tot.fallback, tot.fb_reason[0],
           tot.fb_reason[1], tot.mismatch);
    // wave model: 32x2 tiles (rows are every row_step-th: tile = 32 px x 2 consecutive sampled rows)
    auto wave = [&](const std::vector<int32_t>& it, const char* name) {
        double sum_lock = 0, sum_useful = 0, mx = 0;
        std::vector<double> per;
        for (int ty = 0; ty + 1 < rows; ty += 2)
            for (int tx = 0; tx < W; tx += 32) {
                double wsum = 0;
                for (int b = 0; b < MB; ++b) {
                    int m = 0;
                    for (int yy = 0; yy < 2; ++yy)
                        for (int xx = 0; xx < 32 && tx + xx < W; ++xx) {
                            int v = it[((size_t)(ty + yy) * W + tx + xx) * MB + b];
                            m = std::max(m, v);
                            sum_useful += v;
                        }
                    wsum += m;
                }
                sum_lock += wsum;
                per.push_back(wsum);
                mx = std::max(mx, wsum);
            }
        std::sort(per.begin(), per.end());
        long pmax = 0;
        for (auto& v : it) pmax = std::max<long>(pmax, v);
        printf("%s: lockstep wave-iters total %.3g  SIMD eff %.3f  wave p50 %.0f p99 %.0f p99.9 %.0f max %.0f  max per seg %ld\n",
               name, sum_lock, sum_useful / (64 * sum_lock), per[per.size() / 2], per[per.size() * 99 / 100],
               per[per.size() * 999 / 1000], mx, pmax);
    };
    for (int dd = 0; dd < 40; ++dd)
        if (g_extra[0][dd] + g_extra[1][dd] + g_extra[2][dd] + g_extra[3][dd])
            printf("depth %2d: plain-kept %9ld  margin-kept cone %9ld floor %9ld  unbounded %9ld\n", dd, g_extra[3][dd], g_extra[0][dd], g_extra[1][dd], g_extra[2][dd]);
    wave(it_ref, "ref ");
    wave(it_fast, "fast");
    wave(alu_ref, "ALU ref ");
    wave(alu_fast, "ALU fast");
    return tot.mismatch ? 3 : 0;
}
