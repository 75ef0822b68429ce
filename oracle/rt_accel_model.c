/*
 * rt_accel_model.c — TEST INFRASTRUCTURE ONLY: a CPU model of option
 * "accel"'s walk, built as liboracle_accel.so.  The product
 * never loads it; tests/ and tools/accel_study.py use it as the checker of the
 * accel kernel's work counters and to study how far the accel walk's frames
 * lie from the reference-order oracle (liboracle.so).
 *
 * It is the oracle (rt_oracle.c) with the reference's stack DFS
 * (compute_dynamic_ray.comp:185-210) replaced, through ORC_WALK_HOOK, by the
 * walk the accel kernel runs over the records rt_accel_records returns
 * (3d-ray-tracer-vulkan_amd/csrc/accel_build.h): a ray walks the layout of its
 * direction's octant, slot by slot, next = leaf ? n+2 : (hit ? n+1 : skip),
 * with two rules in place of the reference's compares:
 *   box entered    iff t_exit > t_enter && t_exit > T_MIN &&
 *                  t_enter <= closest_t * (1 + 2^-10) + 2^-10
 *   triangle taken iff t > T_MIN && (t < closest_t || (t == closest_t &&
 *                  flattened index < the current hit's))
 * and one fallback: a segment whose hit lies before its own box's t_enter
 * (t < the leaf's t_enter: rounding on the box face) is walked again with the
 * reference's DFS, counting both walks.  Everything else (camera, scatter,
 * sky, the counters' definitions) is the oracle's own code.  Node visits are
 * box tests (slots walked), as in the reference's counts: 1 + 2 x the internal
 * nodes whose box is entered.
 *
 * orc_accel_format(1): the records are accel_build.h's format 1 (option
 * accel_half): 16-B slots, an internal node one slot with its box in IEEE half
 * precision (decoded exactly, as the kernel's v_cvt_f32_f16), a leaf four.
 */
#define ORC_WALK_HOOK accel_walk
#include "rt_oracle.c"

static const uint32_t* g_rec = NULL;   /* 8 words per slot (format 1: 4) */
static int g_fmt = 0;
static int g_layouts = 1, g_slots = 0, g_root_leaf = 0;
static uint64_t g_fallbacks = 0;       /* segments re-walked in the reference's order */
static uint64_t g_leaf_visits = 0;     /* analysis: leaf slots walked (the rest are internal nodes) */
/* The walk's box margin: a box is entered when t_enter <= closest_t * RELAX +
 * RELAX_ABS (accel_build.h).  orc_accel_margin changes them for studies. */
static float g_relax = 1.0f + 1.0f / 1024.0f, g_relax_abs = 1.0f / 1024.0f;

int orc_accel_margin(float rel, float abs_) {
    g_relax = rel;
    g_relax_abs = abs_;
    return 0;
}

/* Segments re-walked in the reference's order since the last call (resets). */
uint64_t orc_accel_fallbacks(void) {
    const uint64_t f = g_fallbacks;
    g_fallbacks = 0;
    return f;
}

/* Leaf slots walked since the last call (resets); an analysis aid. */
uint64_t orc_accel_leaf_visits(void) {
    const uint64_t f = g_leaf_visits;
    g_leaf_visits = 0;
    return f;
}

/* The format of the records the following renders walk: 0 or 1. */
int orc_accel_format(int fmt) {
    if (fmt != 0 && fmt != 1) return -2;
    g_fmt = fmt;
    return 0;
}

/* An IEEE half (bits h) as float, exactly. */
static float half_to_float(uint32_t h) {
    const uint32_t e = (h >> 10) & 31u, m = h & 1023u;
    float v;
    if (e == 0) v = ldexpf((float)m, -24);
    else if (e == 31) v = m ? NAN : INFINITY;
    else v = ldexpf((float)(1024u + m), (int)e - 25);
    return (h & 0x8000u) ? -v : v;
}

/* Sets the records the following renders walk (the caller keeps them alive). */
int orc_accel_set(const uint32_t* rec, int n_layouts, int slots, int root_leaf) {
    if ((n_layouts != 1 && n_layouts != 8) || slots < 0 || (slots > 0 && !rec)) return -2;
    g_rec = rec;
    g_layouts = n_layouts;
    g_slots = slots;
    g_root_leaf = root_leaf;
    return 0;
}

static float rec_f(size_t slot, int w) {
    float f;
    memcpy(&f, &g_rec[(g_fmt ? 4 : 8) * slot + (size_t)w], 4);
    return f;
}

/* Analysis (orc_accel_quant): internal boxes widened to what a compressed
 * record could hold, to count the visits that would cost; leaves stay exact.
 * 1 = IEEE half precision of each coordinate, rounded outward. */
static int g_quant = 0;
int orc_accel_quant(int mode) { const int o = g_quant; g_quant = mode; return o; }
static float half_down(float x) {           /* the largest half-precision value <= x, as float */
    if (x == 0.0f || !isfinite(x)) return x;
    int E;
    (void)frexpf(x, &E);                     /* |x| in [2^(E-1), 2^E) */
    const int e = E - 1 < -14 ? -14 : E - 1;
    const float ulp = ldexpf(1.0f, e - 10);
    const float r = floorf(x / ulp) * ulp;
    return r > 65504.0f ? 65504.0f : (r < -65504.0f ? -INFINITY : r);
}
static float half_up(float x) { return -half_down(-x); }

static int accel_walk(const scene* s, ray r, float* closest_t, int* hit_index, vec3* hit_normal,
                      orc_counts* cnt) {
    if (g_slots == 0) return 0;                 /* empty scene: every ray misses */
    const int oct = g_layouts == 8 ? ((signbit(r.dir.x) ? 1 : 0) | (signbit(r.dir.y) ? 2 : 0) |
                                      (signbit(r.dir.z) ? 4 : 0)) : 0;
    size_t n = (size_t)oct * (size_t)g_slots;
    const size_t end = n + (size_t)g_slots;
    int leaf = g_root_leaf;
    const vec3 inv = v3(rcp(r.dir.x), rcp(r.dir.y), rcp(r.dir.z));
    float c = *closest_t;
    float thr = c * g_relax + g_relax_abs;
    float hit_te = 0.0f;                      /* t_enter of the hit triangle's own box */
    int hit = -1;
    uint64_t leaf_visits = 0;
    const size_t WS = g_fmt ? 4 : 8;
    while (n < end) {
        const uint32_t aw = g_rec[WS * n + 3], bw = g_fmt ? 0u : g_rec[8 * n + 7];
        cnt->node_visits++;
        trace_rec((int32_t)n);
        /* the slab test of hit_aabb (:88-103), t_enter <= closest_t */
        vec3 blo, bhi;
        if (g_fmt && !leaf) {
            const uint32_t* w = &g_rec[4 * n];
            blo = v3(half_to_float(w[0] & 0xFFFFu), half_to_float(w[0] >> 16), half_to_float(w[1] & 0xFFFFu));
            bhi = v3(half_to_float(w[1] >> 16), half_to_float(w[2] & 0xFFFFu), half_to_float(w[2] >> 16));
        } else {
            blo = v3(rec_f(n, 0), rec_f(n, 1), rec_f(n, 2));
            bhi = v3(rec_f(n, 4), rec_f(n, 5), rec_f(n, 6));
        }
        if (g_quant == 1 && !leaf) {
            blo = v3(half_down(blo.x), half_down(blo.y), half_down(blo.z));
            bhi = v3(half_up(bhi.x), half_up(bhi.y), half_up(bhi.z));
        }
        const vec3 t0s = mul3(sub3(blo, r.origin), inv);
        const vec3 t1s = mul3(sub3(bhi, r.origin), inv);
        const float te = fmaxf(fmaxf(fminf(t0s.x, t1s.x), fminf(t0s.y, t1s.y)), fminf(t0s.z, t1s.z));
        const float tx = fminf(fminf(fmaxf(t0s.x, t1s.x), fmaxf(t0s.y, t1s.y)), fmaxf(t0s.z, t1s.z));
        const int hb = tx > te && tx > T_MIN && te <= thr;
        leaf_visits += (uint64_t)leaf;
        if (hb && leaf) {
            const int tri = (int)(aw & 0x1FFFFFFFu);
            cnt->tri_tests++;
            if ((size_t)tri >= s->n_tris || (size_t)tri >= s->n_mats) return -1;
            /* hit_triangle (:105-129) on the flattened triangle's own vertices */
            vec3 nrm;
            float t = INFINITY;
            if (hit_triangle(r, vertex_pos(s, (size_t)tri * 3 + 0), vertex_pos(s, (size_t)tri * 3 + 1),
                             vertex_pos(s, (size_t)tri * 3 + 2), &t, &nrm) &&
                (t < c || (t == c && tri < hit))) {
                c = t;
                thr = c * g_relax + g_relax_abs;
                hit = tri;
                hit_te = te;
                *hit_normal = nrm;
            }
        }
        size_t nxt;
        int nl;
        if (leaf) {
            nxt = n + (g_fmt ? 4 : 2);
            nl = (int)(aw >> 31);
        } else if (hb) {
            nxt = n + 1;
            nl = g_fmt ? (int)((aw >> 30) & 1u) : (int)(bw & 1u);
        } else {
            nxt = aw & (g_fmt ? 0x3FFFFFFFu : 0x7FFFFFFFu);
            nl = (int)(aw >> 31);
        }
        if (nxt <= n && !hb) return -1;         /* a link that does not move forward: bad records */
        n = nxt;
        leaf = nl;
    }
#ifdef _OPENMP
#pragma omp atomic
#endif
    g_leaf_visits += leaf_visits;
    if (hit >= 0 && c < hit_te) {
        /* The hit lies before its own box's t_enter (float rounding on the
         * box face): the one case where the reference's result depends on
         * its visit order.  Re-walk the segment in the reference's order. */
#ifdef _OPENMP
#pragma omp atomic
#endif
        g_fallbacks++;
        return reference_walk(s, r, closest_t, hit_index, hit_normal, cnt);
    }
    *closest_t = c;
    *hit_index = hit;
    return 0;
}
