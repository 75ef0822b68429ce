/*
 * rt_oracle.c — CPU oracle for the per-pixel path-trace path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * or the timed CPU baseline.  The product (3d-ray-tracer-vulkan_amd/) never
 * links or calls it.
 *
 * A plain-C restatement, line by line, of the reference's executed compute
 * shader shaders/compute_dynamic_ray.comp (byte-identical to
 * compute_with_dynamic_light_source.comp), reading the
 * same std430 buffers the reference uploads: 48-B vertex records
 * (SceneBuilder.java:95-99), 16-B materials (:103), 48-B preorder BVH nodes
 * (BVHFlattener.java:51-97) and the 80-B camera UBO (VulkanEngine.java:387-395).
 * It keeps the reference's own traversal: a DFS with an int stack[64]
 * (compute_dynamic_ray.comp:185-210), not the product's stackless walk.
 *
 * PARITY STATUS: unpinned against a real Vulkan frame.  The reference is
 * Java + GLSL and cannot be built or run here (no JDK, no Vulkan ICD, no
 * glslang); its repository holds no tests or numeric fixtures.
 * This oracle fixes the shader's implementation-defined float behaviour as
 * IEEE binary32 with: no FMA contraction (build with -ffp-contract=off),
 * correctly rounded / and sqrt, normalize(v) = v / sqrt(dot(v,v)),
 * dot = (x*x' + y*y') + z*z', min/max = fminf/fmaxf, reflect(I,N) =
 * I - N*(2*dot(N,I)), and an RGBA8 UNORM store that clamps and rounds to
 * nearest even.  It is cross-checked against an independent numpy
 * restatement (oracle/shader_np.py) and against constants and call order read
 * from the executed SPIR-V (tests/golden/spirv_facts.json).
 *
 * One addition to the reference: randomVec3InUnitSphere's unbounded rejection
 * loop (:65-68) gives up after 65536 triples and returns (0,0,0), where the
 * reference would spin forever; the product kernel has the same bound.
 */
#include "rt_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define T_MIN 0.001f                 /* :42 */
#define T_MAX 10000.0f               /* :43 */
#define MAX_REJECT_TRIPLES 65536
#define STACK_SIZE 64                /* :185 */

/* visit tracing (orc_trace_pixel; analysis aid, single-threaded use only) */
static int32_t* g_trace = NULL;
static int g_trace_cap = 0, g_trace_n = 0;
static void trace_rec(int32_t v) { if (g_trace && g_trace_n < g_trace_cap) g_trace[g_trace_n++] = v; }

typedef struct { float x, y, z; } vec3;

/* Implementation-defined float behaviour.  The default build (liboracle.so)
 * is the contract above: every helper below is the plain IEEE expression.
 * The envelope build (rt_envelope.c, liboracle_env.so; tests/golden/
 * make_envelope.py) switches, per orc_env_set_variant bit, to behaviour a
 * Vulkan implementation is also allowed (GLSL 4.50 §4.7.1, SPIR-V without
 * NoContraction decorations): FMA contraction of a*b+c, normalize through
 * inversesqrt, division through a reciprocal, and approximate (1-ulp)
 * reciprocal / inversesqrt.  It measures how far a real Vulkan frame may lie
 * from the contract. */
#ifdef ORC_ENVELOPE
#define ENV_FMA 1        /* contract a*b+c / a*b-c / c-a*b at the sites LLVM's DAG combiner fuses */
#define ENV_RSQ 2        /* normalize(v) = v * inversesqrt(dot(v,v)), inversesqrt correctly rounded */
#define ENV_RCP 4        /* a / b = a * (1 / b), the reciprocal correctly rounded */
#define ENV_ULP 8        /* reciprocals and inversesqrts off by up to one ulp (a hash of the input picks) */
#define ENV_FTZ 16       /* denormal inputs and results flushed to zero (shaderDenormPreserveFloat32 off) */
#define ENV_ULP2 32      /* reciprocals and inversesqrts off by up to two ulps: with ENV_RCP a division is
                          * within the 2.5 ulps GLSL 4.50 allows, and inversesqrt at its 2-ulp bound */
#define ENV_SQRT_RCP 64  /* sqrt(x) = 1 / inversesqrt(x) (GLSL 4.50 defines sqrt's precision so), at length()
                          * (:139), normalize and the gamma sqrt (:235) */
#define ENV_SQRT_MUL 128 /* sqrt(x) = x * inversesqrt(x) (0 for x = 0), at the same sites */
#include <xmmintrin.h>
static int g_env = 0;
/* the calling thread's SSE control word for the selected variant (FTZ + DAZ or not) */
static void env_fp_mode(void) {
    const unsigned base = _mm_getcsr() & ~0x8040u;
    _mm_setcsr(base | ((g_env & ENV_FTZ) ? 0x8040u : 0u));
}
static float env_ulp(float r, float x) {
    if (!(g_env & (ENV_ULP | ENV_ULP2))) return r;
    uint32_t b;
    memcpy(&b, &x, 4);
    const uint32_t h = orc_pcg(b ^ 0x9E3779B9u);
    if (g_env & ENV_ULP2) {                    /* -2 .. +2 ulps, a hash of the input picks */
        const int k = (int)(h % 5u) - 2;
        for (int i = 0; i < k; ++i) r = nextafterf(r, INFINITY);
        for (int i = 0; i < -k; ++i) r = nextafterf(r, -INFINITY);
        return r;
    }
    const uint32_t h3 = h & 3u;
    return h3 == 1u ? nextafterf(r, INFINITY) : h3 == 2u ? nextafterf(r, -INFINITY) : r;
}
static float mad(float a, float b, float c) { return (g_env & ENV_FMA) ? fmaf(a, b, c) : a * b + c; }
static float msb(float a, float b, float c) { return (g_env & ENV_FMA) ? fmaf(a, b, -c) : a * b - c; }
static float rcp(float x) { return env_ulp(1.0f / x, x); }
static float fdiv(float a, float b) { return (g_env & (ENV_RCP | ENV_ULP | ENV_ULP2)) ? a * rcp(b) : a / b; }
static float rsq(float x) { return env_ulp((float)(1.0 / sqrt((double)x)), x); }
static float fsqrt(float x) {
    if (g_env & ENV_SQRT_RCP) return 1.0f / rsq(x);
    if (g_env & ENV_SQRT_MUL) return x == 0.0f ? 0.0f : x * rsq(x);
    return sqrtf(x);
}
#else
static float mad(float a, float b, float c) { return a * b + c; }
static float msb(float a, float b, float c) { return a * b - c; }
static float rcp(float x) { return 1.0f / x; }
static float fdiv(float a, float b) { return a / b; }
static float fsqrt(float x) { return sqrtf(x); }
#endif

static vec3 v3(float x, float y, float z) { vec3 r = {x, y, z}; return r; }
static vec3 add3(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static vec3 sub3(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static vec3 mul3(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static vec3 scale3(vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
/* a + b * s (add3(a, scale3(b, s)), one contraction site per component) */
static vec3 madd3(vec3 a, vec3 b, float s) { return v3(mad(b.x, s, a.x), mad(b.y, s, a.y), mad(b.z, s, a.z)); }
/* (x*x' + y*y') + z*z'; contracted: fma(z, z', fma(x, x', y*y')) */
static float dot3(vec3 a, vec3 b) { return mad(a.z, b.z, mad(a.x, b.x, a.y * b.y)); }
static float length3(vec3 a) { return fsqrt(dot3(a, a)); }
static vec3 normalize3(vec3 a) {
#ifdef ORC_ENVELOPE
    if (g_env & ENV_RSQ) { const float k = rsq(dot3(a, a)); return v3(a.x * k, a.y * k, a.z * k); }
#endif
    float l = length3(a);
    return v3(fdiv(a.x, l), fdiv(a.y, l), fdiv(a.z, l));
}
static vec3 cross3(vec3 a, vec3 b) {
    return v3(msb(a.y, b.z, a.z * b.y), msb(a.z, b.x, a.x * b.z), msb(a.x, b.y, a.y * b.x));
}
/* I - N * (2 dot(N, I)); contracted: fma(-N, k, I) */
static vec3 reflect3(vec3 i, vec3 n) {
    const float k = 2.0f * dot3(n, i);
    return v3(mad(-n.x, k, i.x), mad(-n.y, k, i.y), mad(-n.z, k, i.z));
}

/* ------------------------------------------------------------------ RNG -- */

uint32_t orc_pcg(uint32_t v) {                                  /* :52-56 */
    uint32_t state = v * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}

float orc_random_float(uint32_t* seed) {                         /* :58-61 */
    *seed = orc_pcg(*seed);
    return (float)(*seed) / (float)0xFFFFFFFFu;
}

static vec3 random_in_unit_sphere(uint32_t* seed) {             /* :63-70 */
    float a = orc_random_float(seed);
    float b = orc_random_float(seed);
    float c = orc_random_float(seed);
    (void)a; (void)b; (void)c;                                  /* temp: drawn, never used */
    for (int it = 0; it < MAX_REJECT_TRIPLES; ++it) {
        float x = orc_random_float(seed);
        float y = orc_random_float(seed);
        float z = orc_random_float(seed);
        vec3 p = v3(msb(x, 2.0f, 1.0f), msb(y, 2.0f, 1.0f), msb(z, 2.0f, 1.0f));
        if (dot3(p, p) < 1.0f) return p;
    }
    return v3(0.0f, 0.0f, 0.0f);
}

void orc_random_in_unit_sphere(uint32_t* seed, float out[3]) {
    vec3 p = random_in_unit_sphere(seed);
    out[0] = p.x; out[1] = p.y; out[2] = p.z;
}

static vec3 random_unit_vector(uint32_t* seed) {                 /* :72-74 */
    return normalize3(random_in_unit_sphere(seed));
}

/* ------------------------------------------------------------- geometry -- */

typedef struct { vec3 origin, dir; } ray;

static vec3 ray_at(ray r, float t) { return madd3(r.origin, r.dir, t); }   /* :77-79 */

static vec3 sky_color(ray r) {                                   /* :81-85 */
    vec3 u = normalize3(r.dir);
    float t = 0.5f * (u.y + 1.0f);
    vec3 one = v3(1.0f, 1.0f, 1.0f);
    return madd3(scale3(one, 1.0f - t), v3(0.5f, 0.7f, 1.0f), t);
}

static int hit_aabb(ray r, vec3 bmin, vec3 bmax, float t_min, float t_max) {    /* :88-103 */
    vec3 inv = v3(rcp(r.dir.x), rcp(r.dir.y), rcp(r.dir.z));
    vec3 t0s = mul3(sub3(bmin, r.origin), inv);
    vec3 t1s = mul3(sub3(bmax, r.origin), inv);
    vec3 tmin = v3(fminf(t0s.x, t1s.x), fminf(t0s.y, t1s.y), fminf(t0s.z, t1s.z));
    vec3 tmax = v3(fmaxf(t0s.x, t1s.x), fmaxf(t0s.y, t1s.y), fmaxf(t0s.z, t1s.z));
    float t_enter = fmaxf(tmin.x, tmin.y);
    t_enter = fmaxf(t_enter, tmin.z);
    float t_exit = fminf(tmax.x, tmax.y);
    t_exit = fminf(t_exit, tmax.z);
    return t_exit > t_enter && t_exit > t_min && t_enter < t_max;
}

static int hit_triangle(ray r, vec3 v0, vec3 v1, vec3 v2,        /* :105-129 */
                        float* closest_t, vec3* hit_normal) {
    vec3 edge1 = sub3(v1, v0);
    vec3 edge2 = sub3(v2, v0);
    vec3 ray_cross_e2 = cross3(r.dir, edge2);
    float det = dot3(edge1, ray_cross_e2);
    if (det > -0.00001f && det < 0.00001f) return 0;
    float inv_det = rcp(det);
    vec3 s = sub3(r.origin, v0);
    float u = inv_det * dot3(s, ray_cross_e2);
    if (u < 0.0f || u > 1.0f) return 0;
    vec3 s_cross_e1 = cross3(s, edge1);
    float v = inv_det * dot3(r.dir, s_cross_e1);
    if (v < 0.0f || (u + v) > 1.0f) return 0;
    float t = inv_det * dot3(edge2, s_cross_e1);
    if (t > T_MIN && t < *closest_t) {
        *closest_t = t;
        *hit_normal = normalize3(cross3(edge1, edge2));
        if (dot3(r.dir, *hit_normal) > 0.0f) *hit_normal = scale3(*hit_normal, -1.0f);
        return 1;
    }
    return 0;
}

/* Extension ORC_EXT_SPHERES (no reference counterpart; the reference is
 * triangles only).  The usual quadratic with half-b,
 * the nearer root first, both against (T_MIN, closest_t); the normal is
 * (p - c) / r, turned to face the ray like hit_triangle's (:125-127). */
static int hit_sphere(ray r, vec3 c, float radius, float* closest_t, vec3* hit_normal) {
    vec3 oc = sub3(r.origin, c);
    float a = dot3(r.dir, r.dir);
    float half_b = dot3(oc, r.dir);
    float cc = dot3(oc, oc) - radius * radius;
    float disc = half_b * half_b - a * cc;
    if (!(disc >= 0.0f)) return 0;
    float sq = sqrtf(disc);
    float root = (-half_b - sq) / a;
    if (!(root > T_MIN && root < *closest_t)) {
        root = (-half_b + sq) / a;
        if (!(root > T_MIN && root < *closest_t)) return 0;
    }
    *closest_t = root;
    vec3 p = ray_at(r, root);
    vec3 n = v3((p.x - c.x) / radius, (p.y - c.y) / radius, (p.z - c.z) / radius);
    if (dot3(r.dir, n) > 0.0f) n = scale3(n, -1.0f);
    *hit_normal = n;
    return 1;
}

/* --------------------------------------------------------------- buffers -- */

static float f32_at(const unsigned char* p, size_t off) { float f; memcpy(&f, p + off, 4); return f; }
static int32_t i32_at(const unsigned char* p, size_t off) { int32_t v; memcpy(&v, p + off, 4); return v; }

typedef struct {
    const unsigned char* verts;   /* 16 B per vertex, 3 per triangle */
    const unsigned char* mats;    /* 16 B per triangle */
    const unsigned char* nodes;   /* 48 B per node */
    size_t n_nodes, n_tris, n_mats;
    const float* spheres;         /* extension ORC_EXT_SPHERES: 8 floats per sphere */
    int n_spheres;
} scene;

static vec3 vertex_pos(const scene* s, size_t i) {
    const unsigned char* p = s->verts + i * 16;
    return v3(f32_at(p, 0), f32_at(p, 4), f32_at(p, 8));
}

static int scatter(const unsigned char* m, uint32_t* seed, ray r_in,   /* :132-154; m = the 16-B material */
                   vec3 hit_pos, vec3 hit_normal, vec3* attenuation, ray* scattered) {
    vec3 albedo = v3(f32_at(m, 0), f32_at(m, 4), f32_at(m, 8));
    float type = f32_at(m, 12);
    if (type == 0.0f) {
        vec3 dir = add3(hit_normal, random_unit_vector(seed));
        if (length3(dir) < 0.0001f) dir = hit_normal;
        scattered->origin = hit_pos;
        scattered->dir = normalize3(dir);
        *attenuation = albedo;
        return 1;
    }
    if (type == 1.0f || type == 2.0f) {
        float fuzz = (type == 2.0f) ? 0.3f : 0.0f;
        vec3 reflected = reflect3(normalize3(r_in.dir), hit_normal);
        vec3 p = random_in_unit_sphere(seed);
        scattered->origin = hit_pos;
        scattered->dir = normalize3(madd3(reflected, p, fuzz));
        *attenuation = albedo;
        return dot3(scattered->dir, hit_normal) > 0.0f;
    }
    return 0;
}

static unsigned char unorm8(float c) {
    return c > 0.0f ? (c < 1.0f ? (unsigned char)rintf(c * 255.0f) : 255) : 0;
}

/* The closest hit of one bounce (:181-210): the reference's DFS with an int
 * stack[64], left child popped first.  Returns 0, or -1 on stack overflow or
 * an out-of-range index (where the reference reads out of bounds). */
static int reference_walk(const scene* s, ray r, float* closest, int* hit_index, vec3* hit_normal,
                          orc_counts* cnt) {
    float closest_t = *closest;
    int hit_triangle_index = *hit_index;
    int stack[STACK_SIZE];
    int sp = 0;
    if (s->n_nodes > 0) stack[sp++] = 0;          /* empty scene: no root to read */
    while (sp > 0) {                                                       /* :189-210 */
        int node_index = stack[--sp];
        if (node_index < 0 || (size_t)node_index >= s->n_nodes) return -1;
        const unsigned char* nd = s->nodes + (size_t)node_index * 48;
        vec3 bmin = v3(f32_at(nd, 0), f32_at(nd, 4), f32_at(nd, 8));
        vec3 bmax = v3(f32_at(nd, 16), f32_at(nd, 20), f32_at(nd, 24));
        int32_t data = i32_at(nd, 32), count = i32_at(nd, 36);
        cnt->node_visits++;
        trace_rec(node_index);
        if (hit_aabb(r, bmin, bmax, T_MIN, closest_t)) {
            if (count < 0) {
                int tri = -(data + 1);
                if (tri < 0 || (size_t)tri >= s->n_tris || (size_t)tri >= s->n_mats) return -1;
                vec3 v0 = vertex_pos(s, (size_t)tri * 3 + 0);
                vec3 v1 = vertex_pos(s, (size_t)tri * 3 + 1);
                vec3 v2 = vertex_pos(s, (size_t)tri * 3 + 2);
                vec3 temp_normal;
                cnt->tri_tests++;
                if (hit_triangle(r, v0, v1, v2, &closest_t, &temp_normal)) {
                    hit_triangle_index = tri;
                    *hit_normal = temp_normal;
                }
            } else {
                if (sp + 2 > STACK_SIZE) return -1;
                stack[sp++] = count;   /* right */
                stack[sp++] = data;    /* left  */
            }
        }
    }
    *closest = closest_t;
    *hit_index = hit_triangle_index;
    return 0;
}

#ifdef ORC_WALK_HOOK
static int ORC_WALK_HOOK(const scene* s, ray r, float* closest_t, int* hit_index, vec3* hit_normal,
                         orc_counts* cnt);
#endif

/* One invocation of main() (:158-237).  Returns 0, or -1 on stack overflow or
 * an out-of-range index (where the reference reads out of bounds). */
static int shade_pixel(const scene* s, const orc_camera* cam, int W, int H, int max_bounces,
                       int px, int py, float out_rgb[3], orc_counts* cnt, uint32_t* prof, int ext,
                       float lin[3]) {
#ifdef ORC_ENVELOPE
    env_fp_mode();
#endif
    uint32_t seed = (uint32_t)(py * W + px);                                   /* :164 */
    if (ext & ORC_EXT_ACCUMULATE)              /* extension: a new sample per frame (frame 0 = :164) */
        seed += (uint32_t)cam->frame_count * (uint32_t)(W * H);
    float u = fdiv((float)px + orc_random_float(&seed), (float)W);             /* :167 */
    float v = fdiv((float)(H - 1 - py) + orc_random_float(&seed), (float)H);   /* :168 */
    vec3 o = v3(cam->origin[0], cam->origin[1], cam->origin[2]);
    vec3 llc = v3(cam->lower_left[0], cam->lower_left[1], cam->lower_left[2]);
    vec3 hor = v3(cam->horizontal[0], cam->horizontal[1], cam->horizontal[2]);
    vec3 ver = v3(cam->vertical[0], cam->vertical[1], cam->vertical[2]);
    ray r;
    r.origin = o;
    r.dir = normalize3(sub3(madd3(madd3(llc, hor, u), ver, v), o));                 /* :173 */

    vec3 final_color = v3(0.0f, 0.0f, 0.0f);
    vec3 attenuation = v3(1.0f, 1.0f, 1.0f);
    for (int b = 0; b < max_bounces; ++b) {                                    /* :179 */
        cnt->segments++;
        trace_rec(-(b + 1));
        const uint64_t nv0 = cnt->node_visits, tt0 = cnt->tri_tests;
        float closest_t = T_MAX;
        int hit_triangle_index = -1;
        vec3 hit_normal = v3(0.0f, 0.0f, 0.0f);
#ifdef ORC_WALK_HOOK
        /* rt_accel_model.c: the accel option's walk instead of the reference's DFS */
        if (ORC_WALK_HOOK(s, r, &closest_t, &hit_triangle_index, &hit_normal, cnt)) return -1;
#else
        if (reference_walk(s, r, &closest_t, &hit_triangle_index, &hit_normal, cnt)) return -1;
#endif
        if (prof) prof[b] = (uint32_t)(cnt->node_visits - nv0) | ((uint32_t)(cnt->tri_tests - tt0) << 20);
        const unsigned char* hit_mat = hit_triangle_index != -1 ? s->mats + (size_t)hit_triangle_index * 16 : NULL;
        if (ext & ORC_EXT_SPHERES) {
            /* extension: after the BVH, every sphere in index order at the closest_t so far */
            for (int k = 0; k < s->n_spheres; ++k) {
                const float* sp_k = s->spheres + 8 * (size_t)k;
                vec3 temp_normal;
                if (hit_sphere(r, v3(sp_k[0], sp_k[1], sp_k[2]), sp_k[3], &closest_t, &temp_normal)) {
                    hit_mat = (const unsigned char*)(sp_k + 4);
                    hit_normal = temp_normal;
                }
            }
        }
        if (hit_mat) {                                                         /* :212 */
            vec3 hit_pos = ray_at(r, closest_t);
            vec3 mat_att;
            ray scattered;
            cnt->mat_reads++;
            if ((ext & ORC_EXT_EMISSIVE) && f32_at(hit_mat, 12) == 3.0f) {
                /* extension: a type-3 material emits its albedo (the reference renders it black) */
                final_color = mul3(attenuation, v3(f32_at(hit_mat, 0), f32_at(hit_mat, 4), f32_at(hit_mat, 8)));
                break;
            }
            if (scatter(hit_mat, &seed, r, hit_pos, hit_normal, &mat_att, &scattered)) {
                attenuation = mul3(attenuation, mat_att);
                r = scattered;
            } else {
                attenuation = v3(0.0f, 0.0f, 0.0f);
                break;
            }
        } else {
            if ((ext & ORC_EXT_SKY_TOGGLE) && cam->sky_enabled == 0)
                final_color = v3(0.0f, 0.0f, 0.0f);   /* extension: sky off, a miss is black */
            else
                final_color = mul3(attenuation, sky_color(r));
            break;
        }
        if (b == max_bounces - 1) final_color = v3(0.0f, 0.0f, 0.0f);         /* :229-231 */
    }
    if (lin) {                                 /* extension: accumulation wants the linear colour */
        lin[0] = final_color.x;
        lin[1] = final_color.y;
        lin[2] = final_color.z;
    }
    out_rgb[0] = fsqrt(final_color.x);                                         /* :235 */
    out_rgb[1] = fsqrt(final_color.y);
    out_rgb[2] = fsqrt(final_color.z);
    return 0;
}

int orc_render(const void* vertices, size_t vertex_bytes,
               const void* materials, size_t material_bytes,
               const void* bvh_nodes, size_t bvh_bytes,
               const orc_camera* cam, int width, int height, int max_bounces,
               int x0, int y0, int tile_w, int tile_h, int row_step,
               uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads) {
    return orc_render_profile(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, bvh_bytes, cam,
                              width, height, max_bounces, x0, y0, tile_w, tile_h, row_step, out_rgba,
                              out_radiance, counts, n_threads, NULL);
}

static int render_core(const void* vertices, size_t vertex_bytes,
               const void* materials, size_t material_bytes,
               const void* bvh_nodes, size_t bvh_bytes,
               const orc_camera* cam, int width, int height, int max_bounces,
               int x0, int y0, int tile_w, int tile_h, int row_step,
               uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads,
               uint32_t* profile, int ext, float* accum, const float* spheres, int n_spheres);

int orc_render_profile(const void* vertices, size_t vertex_bytes,
               const void* materials, size_t material_bytes,
               const void* bvh_nodes, size_t bvh_bytes,
               const orc_camera* cam, int width, int height, int max_bounces,
               int x0, int y0, int tile_w, int tile_h, int row_step,
               uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads,
               uint32_t* profile) {
    return render_core(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, bvh_bytes, cam, width,
                       height, max_bounces, x0, y0, tile_w, tile_h, row_step, out_rgba, out_radiance, counts,
                       n_threads, profile, 0, NULL, NULL, 0);
}

int orc_render_ext(const void* vertices, size_t vertex_bytes,
                   const void* materials, size_t material_bytes,
                   const void* bvh_nodes, size_t bvh_bytes,
                   const orc_camera* cam, int width, int height, int max_bounces,
                   int x0, int y0, int tile_w, int tile_h, int row_step,
                   uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads,
                   int ext, float* accum) {
    if ((ext & ORC_EXT_ACCUMULATE) && !accum) return -2;
    return render_core(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, bvh_bytes, cam, width,
                       height, max_bounces, x0, y0, tile_w, tile_h, row_step, out_rgba, out_radiance, counts,
                       n_threads, NULL, ext, accum, NULL, 0);
}

int orc_render_spheres(const void* vertices, size_t vertex_bytes,
                       const void* materials, size_t material_bytes,
                       const void* bvh_nodes, size_t bvh_bytes,
                       const orc_camera* cam, int width, int height, int max_bounces,
                       int x0, int y0, int tile_w, int tile_h, int row_step,
                       uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads,
                       int ext, float* accum, const float* spheres, int n_spheres) {
    if ((ext & ORC_EXT_ACCUMULATE) && !accum) return -2;
    if (n_spheres < 0 || (n_spheres > 0 && !spheres)) return -2;
    return render_core(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, bvh_bytes, cam, width,
                       height, max_bounces, x0, y0, tile_w, tile_h, row_step, out_rgba, out_radiance, counts,
                       n_threads, NULL, ext, accum, spheres, n_spheres);
}

static int render_core(const void* vertices, size_t vertex_bytes,
               const void* materials, size_t material_bytes,
               const void* bvh_nodes, size_t bvh_bytes,
               const orc_camera* cam, int width, int height, int max_bounces,
               int x0, int y0, int tile_w, int tile_h, int row_step,
               uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads,
               uint32_t* profile, int ext, float* accum, const float* spheres, int n_spheres) {
    if (!cam || width < 1 || height < 1 || max_bounces < 1 || tile_w < 1 || tile_h < 1 ||
        x0 < 0 || y0 < 0 || x0 + tile_w > width || y0 + tile_h > height || row_step < 1)
        return -2;
    scene s;
    s.verts = (const unsigned char*)vertices;
    s.mats = (const unsigned char*)materials;
    s.nodes = (const unsigned char*)bvh_nodes;
    s.n_nodes = bvh_bytes / 48;
    s.n_tris = vertex_bytes / 48;
    s.n_mats = material_bytes / 16;
    s.spheres = spheres;
    s.n_spheres = (ext & ORC_EXT_SPHERES) ? n_spheres : 0;
    const int rows = (tile_h + row_step - 1) / row_step;
    uint64_t seg = 0, nodes = 0, tris = 0, mats = 0;
    int err = 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : seg, nodes, tris, mats) reduction(| : err)
#endif
    for (int rr = 0; rr < rows; ++rr) {
        const int ly = rr * row_step;
        orc_counts c = {0, 0, 0, 0, 0};
        for (int lx = 0; lx < tile_w; ++lx) {
            float rgb[3];
            uint32_t* prof = profile ? profile + ((size_t)rr * (size_t)tile_w + (size_t)lx) * (size_t)max_bounces : NULL;
            if (prof) memset(prof, 0, sizeof(uint32_t) * (size_t)max_bounces);
            float lin[3];
            if (shade_pixel(&s, cam, width, height, max_bounces, x0 + lx, y0 + ly, rgb, &c, prof, ext, lin)) {
                err |= 1;
                rgb[0] = rgb[1] = rgb[2] = 0.0f;
                lin[0] = lin[1] = lin[2] = 0.0f;
            }
            const size_t p = (size_t)rr * (size_t)tile_w + (size_t)lx;
            if (ext & ORC_EXT_ACCUMULATE) {
                /* extension: running sum of the linear colour; shown as sqrt(mean) */
                float* acc = accum + 3 * p;
                const float n = (float)(cam->frame_count + 1);
                for (int k = 0; k < 3; ++k) {
                    acc[k] = cam->frame_count == 0 ? lin[k] : acc[k] + lin[k];
                    rgb[k] = sqrtf(acc[k] / n);
                }
            }
            if (out_rgba) {
                out_rgba[4 * p + 0] = unorm8(rgb[0]);
                out_rgba[4 * p + 1] = unorm8(rgb[1]);
                out_rgba[4 * p + 2] = unorm8(rgb[2]);
                out_rgba[4 * p + 3] = 255;
            }
            if (out_radiance) {
                out_radiance[3 * p + 0] = rgb[0];
                out_radiance[3 * p + 1] = rgb[1];
                out_radiance[3 * p + 2] = rgb[2];
            }
        }
        seg += c.segments; nodes += c.node_visits; tris += c.tri_tests; mats += c.mat_reads;
    }
    if (counts) {
        counts->pixels = (uint64_t)rows * (uint64_t)tile_w;
        counts->segments = seg;
        counts->node_visits = nodes;
        counts->tri_tests = tris;
        counts->mat_reads = mats;
    }
    return err ? -1 : 0;
}

/* Single-function KAT entry points (tests/test_oracle_kat.py). */
int orc_hit_aabb(const float origin[3], const float dir[3], const float bmin[3], const float bmax[3],
                 float t_min, float t_max) {
    ray r;
    r.origin = v3(origin[0], origin[1], origin[2]);
    r.dir = v3(dir[0], dir[1], dir[2]);
    return hit_aabb(r, v3(bmin[0], bmin[1], bmin[2]), v3(bmax[0], bmax[1], bmax[2]), t_min, t_max);
}

int orc_hit_triangle(const float origin[3], const float dir[3], const float v0[3], const float v1[3],
                     const float v2[3], float* closest_t, float normal[3]) {
    ray r;
    r.origin = v3(origin[0], origin[1], origin[2]);
    r.dir = v3(dir[0], dir[1], dir[2]);
    vec3 n = v3(0.0f, 0.0f, 0.0f);
    int h = hit_triangle(r, v3(v0[0], v0[1], v0[2]), v3(v1[0], v1[1], v1[2]), v3(v2[0], v2[1], v2[2]),
                         closest_t, &n);
    normal[0] = n.x; normal[1] = n.y; normal[2] = n.z;
    return h;
}

int orc_hit_sphere(const float origin[3], const float dir[3], const float centre_radius[4],
                   float* closest_t, float normal[3]) {
    ray r;
    r.origin = v3(origin[0], origin[1], origin[2]);
    r.dir = v3(dir[0], dir[1], dir[2]);
    vec3 n = v3(0.0f, 0.0f, 0.0f);
    int h = hit_sphere(r, v3(centre_radius[0], centre_radius[1], centre_radius[2]), centre_radius[3],
                       closest_t, &n);
    normal[0] = n.x; normal[1] = n.y; normal[2] = n.z;
    return h;
}

int orc_scatter(const float material[4], uint32_t* seed, const float dir_in[3],
                const float hit_pos[3], const float normal[3], float att[3], float dir_out[3]) {
    scene s;
    memset(&s, 0, sizeof s);
    s.mats = (const unsigned char*)material;
    s.n_mats = 1;
    ray r_in, sc;
    r_in.origin = v3(0.0f, 0.0f, 0.0f);
    r_in.dir = v3(dir_in[0], dir_in[1], dir_in[2]);
    vec3 a = v3(0.0f, 0.0f, 0.0f);
    sc.origin = v3(0.0f, 0.0f, 0.0f);
    sc.dir = v3(0.0f, 0.0f, 0.0f);
    int ok = scatter(s.mats, seed, r_in, v3(hit_pos[0], hit_pos[1], hit_pos[2]),
                     v3(normal[0], normal[1], normal[2]), &a, &sc);
    att[0] = a.x; att[1] = a.y; att[2] = a.z;
    dir_out[0] = sc.dir.x; dir_out[1] = sc.dir.y; dir_out[2] = sc.dir.z;
    return ok;
}

/* Analysis aid: the node visit sequence of one pixel's path (segment k's
 * visits follow a -(k+1) marker).  Returns the number of entries written, or
 * -1.  Single-threaded; same arithmetic as orc_render. */
int orc_trace_pixel(const void* vertices, size_t vertex_bytes, const void* materials, size_t material_bytes,
                    const void* bvh_nodes, size_t bvh_bytes, const orc_camera* cam, int width, int height,
                    int max_bounces, int px, int py, int32_t* out, int cap) {
    scene s;
    s.verts = (const unsigned char*)vertices;
    s.mats = (const unsigned char*)materials;
    s.nodes = (const unsigned char*)bvh_nodes;
    s.n_nodes = bvh_bytes / 48;
    s.n_tris = vertex_bytes / 48;
    s.n_mats = material_bytes / 16;
    s.spheres = NULL;
    s.n_spheres = 0;
    g_trace = out;
    g_trace_cap = cap;
    g_trace_n = 0;
    orc_counts c = {0, 0, 0, 0, 0};
    float rgb[3];
    int rc = shade_pixel(&s, cam, width, height, max_bounces, px, py, rgb, &c, NULL, 0, NULL);
    g_trace = NULL;
    return rc ? -1 : g_trace_n;
}
