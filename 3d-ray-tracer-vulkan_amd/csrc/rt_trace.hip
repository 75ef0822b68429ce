// rt_trace.hip — gfx950 path-trace kernels for the reference's per-pixel
// render path (shaders/compute_dynamic_ray.comp, dispatched by
// VulkanEngine.recordComputeCommands, VulkanEngine.java:437-515).
//
// Arithmetic contract: every float operation the shader performs is done here
// in IEEE binary32, in the shader's evaluation order, with no contraction
// (built with -ffp-contract=off) and hipcc's correctly rounded f32 division
// and sqrt.  The CPU oracle (oracle/rt_oracle.c) states the same contract, so
// the two agree bit for bit; see DESIGN.md §2.
//
// Traversal: stackless preorder walk over the compact nodes (rt_internal.h),
// which replays the reference's stack DFS (compute_dynamic_ray.comp:185-210)
// node for node: next = hit ? i+1 : skip(i).  Every schedule below visits the
// same nodes, runs the same triangle tests in the same order and sees the same
// closest_t at each test, so frames and work counters are identical.
// Option accel (the default, kFeatAccel) walks the same way over
// a SAH tree built at upload (accel_build.h), in the ray's octant layout, with
// the rules that keep the reference's closest hit (accel_enter, accel_take) and
// the reference-order fallback; kFeatHalf (option accel_half) reads its 16-B
// half-precision internal records; kFeatQ1 / kFeatQ2 (option split_bounce)
// split a frame's paths over two kernels (§4b).
//
// The kernel, trace_simple: one lane = one pixel for its whole path; a wave
// is a tile of 64 pixels (the reference's 8x8 dispatch shape, or 16x4 / 32x2
// / 64x1).  With the cooperative tail, once at most coop_lanes lanes of a wave
// are still walking, the whole wave finishes their walks one ray at a time
// with coop_walk; with a learned heavy-first order the heaviest pixels are
// traced one per wave (heavy_pixel) at the front of the same launch.  A launch
// covers one frame's tile, its interleaved / listed row bands, or the same
// rows of a batch of frames (one camera and output slice each).
//
// Round 3 archived the schedules that measured slower (persistent waves,
// split, tiered, child-pair walk 1, scalar walk 5, LDS top-tree walk 13,
// LDS-DMA walk 14): profiles/r03/archive/README.md.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <rocprim/device/device_scan.hpp>

#include "rt_internal.h"

namespace rtamd {

namespace {

constexpr float kTMin = 0.001f;              // compute_dynamic_ray.comp:42
constexpr float kTMax = 10000.0f;            // :43
constexpr int   kMaxRejectTriples = 1 << 16; // bound on the rejection loop (:65-68), see DESIGN.md

struct V3 { float x, y, z; };

__device__ __forceinline__ V3 vadd(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 vsub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 vmul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ V3 vscale(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float vdot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ V3 vcross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ V3 vnormalize(V3 a) {
    const float l = sqrtf(vdot(a, a));
    return {a.x / l, a.y / l, a.z / l};
}

// pcg (compute_dynamic_ray.comp:52-56) and randomFloat (:58-61).
__device__ __forceinline__ uint32_t pcg(uint32_t v) {
    const uint32_t s = v * 747796405u + 2891336453u;
    const uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}
__device__ __forceinline__ float rnd(uint32_t& seed) {
    seed = pcg(seed);
    return (float)seed / 4294967296.0f;   // float(0xFFFFFFFFu) rounds to 2^32
}

// randomVec3InUnitSphere (:63-70): three draws are made and discarded, then
// rejection sampling of 2*rand3-1 until dot(p,p) < 1.
__device__ __forceinline__ V3 rnd_in_sphere(uint32_t& seed) {
    seed = pcg(pcg(pcg(seed)));
    for (int it = 0; it < kMaxRejectTriples; ++it) {
        const float a = rnd(seed);
        const float b = rnd(seed);
        const float c = rnd(seed);
        const V3 p = {a * 2.0f - 1.0f, b * 2.0f - 1.0f, c * 2.0f - 1.0f};
        if (vdot(p, p) < 1.0f) return p;
    }
    return {0.0f, 0.0f, 0.0f};
}

__device__ __forceinline__ uint8_t unorm8(float c) {
    // VkFormat R8G8B8A8_UNORM store: clamp to [0,1], round to nearest even.
    return c > 0.0f ? (c < 1.0f ? (uint8_t)__builtin_rintf(c * 255.0f) : (uint8_t)255) : (uint8_t)0;
}

// Frame row of local row ly of frame f of the launch (rt_internal.h, TraceArgs
// band mapping; the caller skips a per-frame list's -1 padding entries).
__device__ __forceinline__ int frame_row(const TraceArgs& a, int f, int ly) {
    if (a.band_list) return a.y0 + a.band_list[f * a.list_stride + ly / a.band_h] * a.band_h + ly % a.band_h;
    return a.y0 + ((ly / a.band_h) * a.band_stride + a.band_off) * a.band_h + ly % a.band_h;
}

// Seed, AA jitter and primary ray (:164-173) of frame f of the launch.
__device__ __forceinline__ void primary_ray_seeded(const TraceArgs& a, int f, int x, int y, uint32_t& seed, V3& o,
                                                   V3& d);
__device__ __forceinline__ void primary_ray(const TraceArgs& a, int f, int x, int y, uint32_t& seed, V3& o, V3& d) {
    seed = (uint32_t)(y * a.width + x);
    primary_ray_seeded(a, f, x, y, seed, o, d);
}

// primary_ray with a caller-chosen initial seed (the accumulation extension).
__device__ __forceinline__ void primary_ray_seeded(const TraceArgs& a, int f, int x, int y, uint32_t& seed, V3& o,
                                                   V3& d) {
    const float u = ((float)x + rnd(seed)) / (float)a.width;
    const float v = ((float)(a.height - 1 - y) + rnd(seed)) / (float)a.height;
    const CamF& c = a.cams[f];                 // f is wave-uniform: scalar loads of the kernel argument
    const V3 cam_o = {c.ox, c.oy, c.oz};
    const V3 cam_l = {c.lx, c.ly, c.lz};
    const V3 cam_h = {c.hx, c.hy, c.hz};
    const V3 cam_v = {c.vx, c.vy, c.vz};
    o = cam_o;
    d = vnormalize(vsub(vadd(vadd(cam_l, vscale(cam_h, u)), vscale(cam_v, v)), cam_o));
}

// Slab test of hit_aabb (:88-103), split into the part that does not depend
// on closest_t (ind) and t_enter; the box is hit iff ind && te < closest_t.
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void slab(float4 A, float4 B, V3 o, V3 inv, float& te, bool& ind) {
    // x and y in packed FP32 (v_pk_add_f32 / v_pk_mul_f32: two IEEE binary32
    // operations per lane per instruction, each rounded exactly as the scalar one).
    const f2 oxy = {o.x, o.y}, ixy = {inv.x, inv.y};
    const f2 t0 = (f2{A.x, A.y} - oxy) * ixy;
    const f2 t1 = (f2{B.x, B.y} - oxy) * ixy;
    const float t0x = t0.x, t1x = t1.x, t0y = t0.y, t1y = t1.y;
    const float t0z = (A.z - o.z) * inv.z, t1z = (B.z - o.z) * inv.z;
    te = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tx = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    ind = tx > te && tx > kTMin;
}

// hit_triangle (:105-129) up to its final "t < closest_t" compare: returns
// true and t when det, u, v and t > T_MIN all pass.
__device__ __forceinline__ bool tri_test(float4 P0, float4 P1, float4 P2, V3 o, V3 d, float& t) {
    const V3 v0 = {P0.x, P0.y, P0.z};
    const V3 e1 = {P1.x, P1.y, P1.z};
    const V3 e2 = {P2.x, P2.y, P2.z};
    const V3 pv = vcross(d, e2);
    const float det = vdot(e1, pv);
    if (det > -0.00001f && det < 0.00001f) return false;
    const float inv_det = 1.0f / det;
    const V3 s = vsub(o, v0);
    const float uu = inv_det * vdot(s, pv);
    if (uu < 0.0f || uu > 1.0f) return false;
    const V3 q = vcross(s, e1);
    const float vv = inv_det * vdot(d, q);
    if (vv < 0.0f || (uu + vv) > 1.0f) return false;
    t = inv_det * vdot(e2, q);
    return t > kTMin;
}

// Keep loaded values where they are: an empty asm that "modifies" them stops
// the compiler from sinking a load into the branch that uses it (which would
// turn one memory round trip into two dependent ones).
__device__ __forceinline__ void pin(float4& q) { asm volatile("" : "+v"(q.x), "+v"(q.y), "+v"(q.z), "+v"(q.w)); }

// One node of the walk.  `leaf` says whether node i is a leaf (from its
// predecessor's L bits), so the leaf's triangle is fetched in the same round
// trip as the node.  Returns the next node index and updates `leaf`.
//
// Visit counting, in every walk: the reference's DFS pushes the root once and
// both children of every internal node whose box is hit, and pops (= visits)
// every node it pushes, so a segment visits exactly 1 + 2 x (hit internal
// nodes) nodes.  Walks count the root when the segment starts and 2 per hit
// internal node, which lets a walk skip children it can prove are missed
// without visiting them.
template <bool COUNT>
__device__ __forceinline__ int node_step(const float4* __restrict__ nodes, const float4* __restrict__ leafs,
                                         int i, bool& leaf, V3 o, V3 d, V3 inv, float& closest, int& hit,
                                         unsigned long long& c_node, unsigned long long& c_tri) {
    const float4 A = nodes[2 * i];
    const float4 B = nodes[2 * i + 1];
    // Read only when `leaf`: left undefined otherwise, so the compiler does
    // not zero twelve registers on every step.
    float4 P0, P1, P2;
    if (leaf) {
        P0 = leafs[3 * i + 0];
        P1 = leafs[3 * i + 1];
        P2 = leafs[3 * i + 2];
        pin(P0);   // three whole 16-B loads, not five partial ones
        pin(P1);
        pin(P2);
    }
    float te;
    bool ind;
    slab(A, B, o, inv, te, ind);
    const bool hb = ind && te < closest;
    if (COUNT && hb && !leaf) c_node += 2;
    if (hb && leaf) {
        if (COUNT) ++c_tri;
        float t;
        if (tri_test(P0, P1, P2, o, d, t) && t < closest) {
            closest = t;
            hit = __float_as_int(P0.w);
        }
    }
    const uint32_t aw = __float_as_uint(A.w), bw = __float_as_uint(B.w);
    leaf = hb ? (bw & 1u) : (aw >> 31);
    return hb ? i + 1 : (int)(aw & 0x7FFFFFFFu);
}

// The hit normal of :124-125: normalize(cross(e1,e2)) (precomputed per
// triangle, rt_internal.h), flipped to face against d.
__device__ __forceinline__ V3 hit_normal(const float4* __restrict__ norms, int hit, V3 d) {
    const float4 N = norms[kShadeStride * hit];
    V3 n = {N.x, N.y, N.z};
    if (vdot(d, n) > 0.0f) n = {-n.x, -n.y, -n.z};
    return n;
}

// Extension kExtSpheres (no reference counterpart; oracle/rt_oracle.h
// ORC_EXT_SPHERES states the same arithmetic): after the BVH walk, every
// sphere in index order against (T_MIN, closest); a hit sets hit = -2 - k.
// The sphere index is wave-uniform, so every lane reads the same record.
__device__ __forceinline__ void sphere_tests(const float4* __restrict__ sph, int n, V3 o, V3 d,
                                             float& closest, int& hit) {
    const float qa = vdot(d, d);
    for (int k = 0; k < n; ++k) {
        const float4 S = sph[2 * k];
        const V3 oc = {o.x - S.x, o.y - S.y, o.z - S.z};
        const float hb = vdot(oc, d);
        const float qc = vdot(oc, oc) - S.w * S.w;
        const float disc = hb * hb - qa * qc;
        if (!(disc >= 0.0f)) continue;
        const float sq = sqrtf(disc);
        float root = (-hb - sq) / qa;
        if (!(root > kTMin && root < closest)) {
            root = (-hb + sq) / qa;
            if (!(root > kTMin && root < closest)) continue;
        }
        closest = root;
        hit = -2 - k;
    }
}

// The sphere normal (p - c) / r at the hit point, turned to face against d.
__device__ __forceinline__ V3 sphere_normal(float4 S, V3 hp, V3 d) {
    V3 n = {(hp.x - S.x) / S.w, (hp.y - S.y) / S.w, (hp.z - S.z) / S.w};
    if (vdot(d, n) > 0.0f) n = {-n.x, -n.y, -n.z};
    return n;
}

// scatter (:132-154).  Returns true and the new direction on scatter.
__device__ __forceinline__ bool scatter(float4 M, V3 d, V3 n, uint32_t& seed, V3& nd) {
    if (M.w == 0.0f) {                                                    // Lambertian :137-143
        const V3 ru = vnormalize(rnd_in_sphere(seed));
        V3 sd = vadd(n, ru);
        if (sqrtf(vdot(sd, sd)) < 0.0001f) sd = n;
        nd = vnormalize(sd);
        return true;
    }
    if (M.w == 1.0f || M.w == 2.0f) {                                     // metal :145-151
        const float fuzz = (M.w == 2.0f) ? 0.3f : 0.0f;
        const V3 di = vnormalize(d);
        const float k = 2.0f * vdot(n, di);
        const V3 refl = vsub(di, vscale(n, k));                           // reflect()
        const V3 p = rnd_in_sphere(seed);
        nd = vnormalize(vadd(refl, vscale(p, fuzz)));
        return vdot(nd, n) > 0.0f;
    }
    nd = d;
    return false;                                                         // :153
}

__device__ __forceinline__ V3 sky_color(V3 d) {                          // getSkyColor :81-85
    const V3 ud = vnormalize(d);
    const float t = 0.5f * (ud.y + 1.0f);
    const float omt = 1.0f - t;
    return {omt * 1.0f + t * 0.5f, omt * 1.0f + t * 0.7f, omt * 1.0f + t * 1.0f};
}

__device__ __forceinline__ void write_pixel(const TraceArgs& a, int lx, int ly, V3 fin) {
    const V3 g = {sqrtf(fin.x), sqrtf(fin.y), sqrtf(fin.z)};              // :235
    const size_t p = (size_t)ly * (size_t)a.tw + (size_t)lx;
    if (a.out_rgba) a.out_rgba[p] = make_uchar4(unorm8(g.x), unorm8(g.y), unorm8(g.z), 255);
    if (a.out_rad) {
        a.out_rad[3 * p + 0] = g.x;
        a.out_rad[3 * p + 1] = g.y;
        a.out_rad[3 * p + 2] = g.z;
    }
}

constexpr int kFeatExtBit = 16;   // = kFeatExt (defined with the other feature flags below)

// The end of a path: (extension) the accumulation of the linear colour,
// then the sqrt'd RGBA8 store (:235).
template <int FEAT>
__device__ __forceinline__ void finish_pixel(const TraceArgs& a, int lx, int ly, V3 fin) {
    if ((FEAT & kFeatExtBit) && (a.ext & kExtAccumulate)) {
        // extension: running sum of the linear colour, shown as sqrt(mean)
        float* acc = a.accum + 3 * ((size_t)ly * (size_t)a.tw + (size_t)lx);
        const float nf = (float)(a.frame_count + 1);
        const V3 sum = a.frame_count == 0 ? fin : V3{acc[0] + fin.x, acc[1] + fin.y, acc[2] + fin.z};
        acc[0] = sum.x;
        acc[1] = sum.y;
        acc[2] = sum.z;
        fin = {sum.x / nf, sum.y / nf, sum.z / nf};
    }
    write_pixel(a, lx, ly, fin);
}

__device__ __forceinline__ void flush_counters(Counters* c, unsigned long long s, unsigned long long n,
                                               unsigned long long t, unsigned long long m) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        s += __shfl_xor(s, off);
        n += __shfl_xor(n, off);
        t += __shfl_xor(t, off);
        m += __shfl_xor(m, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&c->segments, s);
        atomicAdd(&c->node_visits, n);
        atomicAdd(&c->tri_tests, t);
        atomicAdd(&c->mat_reads, m);
    }
}

__device__ __forceinline__ int lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}


__device__ __forceinline__ int lane_i(int v, int k) { return __builtin_amdgcn_readlane(v, k); }

// Lane k + 1's value in lane k (DPP wave_shl:1; lane 63 keeps its own).
__device__ __forceinline__ float next_lane(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x130, 0xf, 0xf, false));
}
__device__ __forceinline__ float4 next_lane(float4 v) {
    return make_float4(next_lane(v.x), next_lane(v.y), next_lane(v.z), next_lane(v.w));
}

// Bits [0, n) of a wave mask (n in 0..64).
__device__ __forceinline__ uint64_t lanes_lt(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }

// Exclusive prefix max over the wave's lanes (lane 0 gets -1): DPP row
// shifts, row broadcasts, then a one-lane wave shift.
__device__ __forceinline__ int wave_excl_max(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return __builtin_amdgcn_update_dpp(-1, v, 0x138, 0xf, 0xf, false);        // wave_shr:1
}
__device__ __forceinline__ float lane_f(float v, int k) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

// Option accel's rules (accel_build.h).  A box is entered when
// t_enter <= closest_t * (1 + 2^-10) + 2^-10: every box holding a triangle
// that ties or beats closest_t is entered, even where rounding puts the
// triangle's t a little before its box's t_enter.  A triangle is taken on
// t < closest_t, or on a tie with a lower flattened index (the reference
// visits leaves in flattened-index order and keeps the first hit at a given
// t).  oracle/rt_accel_model.c states the same arithmetic.
//
// Thin triangles (round 6; accel_build.h accel_class): Moeller-Trumbore's t
// error grows as 1 / sin of the triangle's angle at v0, so a record whose
// subtree holds a triangle of shape class >= 7 (bit 29 of its link word,
// kAccelForce; a leaf: its own triangle) is entered whenever its slab test
// passes, whatever closest_t.  The rest keep the 2^-10 margin.  Nothing else
// changes: a forced record only enters more boxes.  (Per-record factors, R =
// 1 + 2^(c - 16) in word 7, measured 5% slower on config 3 for the VALU of
// choosing and applying them on every step: profiles/r06/r6h.)
constexpr float kRelax = 1.0f + 1.0f / 1024.0f;
constexpr float kRelaxAbs = 1.0f / 1024.0f;
constexpr uint32_t kThinLeaf = 1u << 29;     // format 1 / 2 leaves: a thin triangle
constexpr uint32_t kForce = 1u << 29;        // format 0: accel_build.h kAccelForce
constexpr uint32_t kIdx = 0x1FFFFFFFu;       // node index bits of a link word (bit 29: kForce)
constexpr uint32_t kTri = 0x1FFFFFFFu;       // triangle index bits of a leaf's link word (bit 29: pad after
                                             //   it on the reference's tree, kForce on option accel's)
__device__ __forceinline__ bool accel_enter(float te, float closest) { return te <= closest * kRelax + kRelaxAbs; }
// (A/B builds: RT_THIN_MARGIN 0 = round 5's rule, the 2^-10 margin
// everywhere, not exact for thin triangles: make variant NAME=x
// FLAGS=-DRT_THIN_MARGIN=0)
#ifndef RT_THIN_MARGIN
#define RT_THIN_MARGIN 1
#endif
// Format 0's entry rule for a record with link word aw.
__device__ __forceinline__ bool accel_enter_w(float te, float closest, uint32_t aw) {
#if RT_THIN_MARGIN
    return accel_enter(te, closest) || (aw & kForce) != 0u;
#else
    (void)aw;
    return accel_enter(te, closest);
#endif
}
// The same with the bound closest_t * (1 + 2^-10) + 2^-10 (the same two
// roundings) kept in lim, recomputed only when closest_t changes: the per-node
// walk's form (two VALU instructions fewer per step).
__device__ __forceinline__ float accel_lim(float closest) { return closest * kRelax + kRelaxAbs; }
__device__ __forceinline__ bool accel_enter_lim(float te, float lim, uint32_t aw) {
#if RT_THIN_MARGIN
    return te <= lim || (aw & kForce) != 0u;
#else
    (void)aw;
    return te <= lim;
#endif
}
__device__ __forceinline__ bool accel_enter_r(float te, float closest, float r) {
    return te <= closest * r + kRelaxAbs;
}
__device__ __forceinline__ bool accel_take(float t, int tri, float closest, int hit) {
    return t < closest || (t == closest && tri < hit);
}

// ------------------------------------------------------------ cooperative walk --
#ifndef RT_CHAIN
// The lockstep walk's next records: 2 = buffer loads whose address is one
// shift of the slot index (config 3 0.2947-0.2960 vs 0.2965-0.2980 ms, config 5
// 8.07-8.10 vs 8.10-8.11, profiles/r04/r4s abchain; records < 4 GB, checked at
// upload); 3 = the same with two selects (equal: 0.2957-0.2963 vs
// 0.2955-0.2977, profiles/r04/r4v); 1 = one select on the chain with global
// loads (slower: 0.298-0.300, 8.42-8.56); 0 = global loads.
#define RT_CHAIN 2
#endif
#ifndef RT_COOP_BUF
// 1 = cooperative windows through buffer loads: slower (config 3 0.2969-0.2986 vs
// 0.2946-0.2957 ms; 8 B more scratch per lane; profiles/r04/r4y), so 0
#define RT_COOP_BUF 0
#endif
#if RT_COOP_BUF
__device__ __forceinline__ float4 wbuf_s(__amdgpu_buffer_rsrc_t r, int voff, unsigned soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, (int)soff, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
#endif
#if RT_CHAIN >= 2
__device__ __forceinline__ float4 wbuf(__amdgpu_buffer_rsrc_t r, int slot, int off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)((unsigned)slot << 5) + off, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
// the same at a byte offset (slot << 5) the caller already holds
__device__ __forceinline__ float4 wbuf_b(__amdgpu_buffer_rsrc_t r, unsigned byte, int off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte + off, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
#endif
#ifndef RT_ACC_SCALAR
// 1 = a walk step whose walking lanes all go to one slot loads it through the
// scalar cache (one s_load per 16 B, no vector-memory issue); A/B builds
#define RT_ACC_SCALAR 0
#endif
// 16-B piece k of the walk records through the scalar cache: k must be
// wave-uniform (readfirstlane), the records read-only for the kernel's life.
__device__ __forceinline__ float4 sbuf(const float4* base, int k) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(4))) const v4f cv4f;
    const v4f v = reinterpret_cast<cv4f*>(reinterpret_cast<uintptr_t>(base))[k];
    return make_float4(v[0], v[1], v[2], v[3]);
}
// A half-format accel record's 16-B slot (accel_build.h format 1).
__device__ __forceinline__ float4 hbuf(__amdgpu_buffer_rsrc_t r, int slot) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)((unsigned)slot << 4), 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
// The low / high IEEE half of a word, as float (exact).
__device__ __forceinline__ float half_lo(uint32_t w) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xFFFFu));
}
__device__ __forceinline__ float half_hi(uint32_t w) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16));
}
#ifndef RT_COOP_DPP
#define RT_COOP_DPP 1      // a leaf's triangle from the next lane by DPP (0: loaded by the lane, A/B builds)
#endif
//
// The whole wave walks ONE ray (arguments wave-uniform), replaying the
// reference's visit sequence exactly:
//   1. lane k < WIN loads slot n+k of the window [n, n+WIN) of the walk records
//      (DevScene::walk): 2 coalesced 16-B loads per lane.  A leaf's triangle is
//      the slot after its box, which lane k+1 loaded: it comes across by DPP
//      (wave_shl:1), so a window costs 2 loads, not 4 (bit 30 of the link word
//      says leaf; a leaf's second slot is loaded as a node nobody visits).  A
//      leaf in slot 63, whose triangle lies past the window, starts the next
//      window instead.  Each lane runs the slab test and, for a leaf whose box
//      is hit at the current closest_t, the triangle test up to "t < closest_t";
//   2. ballots make 64-bit masks: box hit at closest_t (H), triangle hit that
//      improves closest_t (T), is a leaf (Lf);
//   3. the scalar unit replays the walk through the window: the node at slot
//      k is hit iff bit k of H; next = k+1 (an internal node hit), k+2 (a
//      leaf, hit or not), skip(k) (an internal node missed); a triangle hit
//      updates closest_t / hit and re-ballots H and T (closest_t only shrinks,
//      so a leaf not pre-tested at the old closest_t cannot hit at the new one).
// The float operations are node_step's, so closest_t, the hit and the visit /
// triangle-test counts equal the per-lane walk's.
// WIN = 64 slots, or 32 (option coop_window; kFeatWin32): a window serves 4.2
// visits on average in config 5's tails (median 2) and uses 2.5 of its ~17
// lines (tools/layout_model.py); half a window costs ~22% more windows there and
// fetches ~35% fewer lines.
// PAD: the records may hold pad slots (leaf_align; the kernel's kFeatPad).
// ACC: option accel's records and rules (accel_enter / accel_take); `incons`
// tracks whether the hit lies before its own box's t_enter.
template <bool COUNT, int WIN = 64, bool PAD = true, bool ACC = false>
__device__ __forceinline__ int coop_walk(const float4* __restrict__ walk, int end, int n, V3 o, V3 d, V3 inv,
                                         float& closest, int& hit, unsigned long long& c_node,
                                         unsigned long long& c_tri, bool& incons) {
    const int lane = threadIdx.x & 63;
    int windows = 0;
#if RT_COOP_BUF
    // buffer loads: lane k's offset k x 32 B is fixed, the window start is the
    // scalar offset, so no vector instruction sits between the replay's next n
    // and the window's loads
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float4*>(walk), 0, (int)((unsigned)(end + 2) * 32u), 0x00020000);
    const int voff = lane << 5;
#endif
    while (n < end) {
        ++windows;
        const int j = n + lane;
        const bool ld = j < end && lane < WIN;
        float te = 0.0f, tt = 0.0f;
        uint32_t law = 0u;                                           // ACC: the record's link word (kForce)
        int sk = 0, tri = -1;
        bool ind = false, tv = false, lf = false, pd = false;
        float4 A = make_float4(0.f, 0.f, 0.f, 0.f), B = A;
#if RT_COOP_DPP
#if RT_COOP_BUF
        if (ld) {                                                   // window start in the scalar offset
            A = wbuf_s(rs, voff, (unsigned)n << 5);
            B = wbuf_s(rs, voff + 16, (unsigned)n << 5);
        }
#else
        if (ld) {
            A = walk[2 * j];
            B = walk[2 * j + 1];
        }
#endif
        const float4 Q0 = next_lane(A), Q1 = next_lane(B);          // the slot after this one (every lane active)
#else
        float4 Q0 = A, Q1 = A;                                       // (A/B variant: the slot after, loaded)
        if (ld) {
            A = walk[2 * j];
            B = walk[2 * j + 1];
            Q0 = walk[2 * j + 2];
            Q1 = walk[2 * j + 3];
        }
#endif
        if (ld) {
            slab(A, B, o, inv, te, ind);
            const uint32_t aw = __float_as_uint(A.w);
            lf = ((aw >> 30) & 1u) != 0u;
            // a leaf's skip is its successor, two slots on (three past a pad slot)
            // (the code generated for these lines moves the frame time by
            // several percent: written with masks the PAD form measured 2.7%
            // slower on config 3, profiles/r04/r4n)
            if (PAD) {
                sk = lf ? j + 2 + (int)((aw >> 29) & 1u) : (int)(aw & kIdx);
                pd = lf ? ((aw >> 29) & 1u) != 0u : ((__float_as_uint(B.w) >> 2) & 1u) != 0u;
            } else {
                sk = lf ? j + 2 : (int)(aw & kIdx);
            }
            tri = (int)(aw & kTri);
            if (ACC) law = aw;
            if (lf && ind && (ACC ? accel_enter_w(te, closest, aw) : te < closest) && (!RT_COOP_DPP || lane < WIN - 1))
                tv = tri_test(make_float4(B.w, Q0.x, Q0.y, 0.f), make_float4(Q0.z, Q0.w, Q1.x, 0.f),
                              make_float4(Q1.y, Q1.z, Q1.w, 0.f), o, d, tt);
        }
        uint64_t H = __ballot(ind && (ACC ? accel_enter_w(te, closest, law) : te < closest));
        uint64_t T = __ballot(tv && (ACC ? accel_take(tt, tri, closest, hit) : tt < closest));
        const uint64_t Lf = __ballot(lf);
        const uint64_t Pd = PAD ? __ballot(pd) : 0ull;              // a pad slot follows (leaf alignment)
        int lim = min(WIN, end - n);
        if (RT_COOP_DPP && lim == WIN && ((Lf >> (WIN - 1)) & 1ull))
            lim = WIN - 1;                                   // its triangle is past the window
        int k = 0;
        while (k < lim) {
            if ((H >> k) & 1ull) {
                if (COUNT && !((Lf >> k) & 1ull)) c_node += 2;
                if ((Lf >> k) & 1ull) {
                    if (COUNT) ++c_tri;
                    if ((T >> k) & 1ull) {
                        closest = lane_f(tt, k);
                        hit = lane_i(tri, k);
                        if (ACC) incons = closest < lane_f(te, k);
                        H = __ballot(ind && (ACC ? accel_enter_w(te, closest, law) : te < closest));
                        T = __ballot(tv && (ACC ? accel_take(tt, tri, closest, hit) : tt < closest));
                    }
                }
                if (PAD)
                    k += (((Lf >> k) & 1ull) ? 2 : 1) + (int)((Pd >> k) & 1ull);
                else
                    k += ((Lf >> k) & 1ull) ? 2 : 1;
            } else {
                k = lane_i(sk, k) - n;
            }
        }
        n += k;
    }
    return windows;
}

// ------------------------------------------------------------ wide walk --
//
// Option accel_wide (accel_build.h format 2; oracle/rt_accel_model.c
// wide_walk states the same walk on the CPU).  One step per lockstep
// iteration: the lane reads the 48 bytes of the record its link names
// (three 16-B buffer loads).
//   * A leaf: hit_triangle on v0 / e1 / e2; only a hit the walk would take
//     (accel_take) reads the last 16 bytes (the rest of the leaf's exact box)
//     and runs the reference's slab test with the leaf's rule, which decides.
//   * A wide node: each child's box decoded from the node's grid (origin +
//     q 2^e, exactly the host's float arithmetic, so the decoded box holds
//     the child's true box) and slab-tested with the child's rule; the
//     entered children in (t_enter, slot) order: the first is next, the
//     others go on the lane's stack, farthest first.
// Then (a leaf, or no child entered) the lane pops: an entry whose box would
// no longer be entered is dropped (default-margin entries; t_enter kept as
// bfloat16 rounded down, so a drop is always right).  An empty stack ends
// the walk; a push past kWideStackK entries marks the segment for the
// reference-order fallback (wovf).  The stack: kWideStackK x 64 links (4 B)
// then kWideStackK x 64 bfloat16 t_enter (2 B) per wave in LDS, entry k of
// lane l at k x 64 + l (no bank conflicts).
constexpr uint32_t kWLeaf = 1u << 31, kWThin = 1u << 30, kWWider = 1u << 29, kWIdx = 0x07FFFFFFu;
constexpr int kWideStackK = 12;     // accel_build.h kWideStack: 2e-5 of config 3's segments overflow (model)

__device__ __forceinline__ float4 wrec(__amdgpu_buffer_rsrc_t r, int off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

// One step of the wide walk; returns whether the lane still walks.
template <bool COUNT>
__device__ __forceinline__ bool wide_step(__amdgpu_buffer_rsrc_t wrs, uint4* stk, V3 o, V3 d, V3 inv, float& closest,
                                          int& hit, bool& incons, uint32_t& cur, int& sp, bool& ovf,
                                          unsigned long long& c_node, unsigned long long& c_tri) {
    const int lane = threadIdx.x & 63;
    uint32_t* sl = reinterpret_cast<uint32_t*>(stk);                                 // links
    unsigned short* st = reinterpret_cast<unsigned short*>(sl + kWideStackK * 64);   // bfloat16 t_enter
    const int off = (int)((cur & kWIdx) << 6);
    const float4 R0 = wrec(wrs, off), R1 = wrec(wrs, off + 16), R2 = wrec(wrs, off + 32);
    bool pop = true;
    if (cur & kWLeaf) {
        if (COUNT) ++c_tri;
        const uint32_t w0 = __float_as_uint(R0.x);
        const int tri = (int)(w0 & 0x1FFFFFFFu);
        float t;
        if (tri_test(make_float4(R0.y, R0.z, R0.w, 0.f), make_float4(R1.x, R1.y, R1.z, 0.f),
                     make_float4(R2.x, R2.y, R2.z, 0.f), o, d, t) &&
            accel_take(t, tri, closest, hit)) {
            const float4 R3 = wrec(wrs, off + 48);
            if (COUNT) ++c_node;
            float te;
            bool ind;
            slab(make_float4(R1.w, R2.w, R3.x, 0.f), make_float4(R3.y, R3.z, R3.w, 0.f), o, inv, te, ind);
            if (ind && accel_enter_r(te, closest, (w0 & kThinLeaf) ? __builtin_inff() : kRelax)) {
                closest = t;
                hit = tri;
                incons = t < te;
            }
        }
    } else {
        const uint32_t w3 = __float_as_uint(R0.w);
        const int n = (int)((w3 >> 24) & 7u);
        const float sx = __builtin_ldexpf(1.0f, (int)(int8_t)(w3 & 0xFFu));
        const float sy = __builtin_ldexpf(1.0f, (int)(int8_t)((w3 >> 8) & 0xFFu));
        const float sz = __builtin_ldexpf(1.0f, (int)(int8_t)((w3 >> 16) & 0xFFu));
        const uint32_t qlx = __float_as_uint(R1.x), qly = __float_as_uint(R1.y), qlz = __float_as_uint(R1.z);
        const uint32_t qhx = __float_as_uint(R1.w), qhy = __float_as_uint(R2.x), qhz = __float_as_uint(R2.y);
        const uint32_t w10 = __float_as_uint(R2.z), fl = __float_as_uint(R2.w);
        const int cls = (int)(w10 >> 27);
        const float nr = cls < 7 ? kRelax : 1.0f + __builtin_ldexpf(1.0f, cls - 16);
        const uint32_t base = w10 & kWIdx;
        if (COUNT) c_node += (unsigned long long)n;
        // the children's (t_enter, slot) keys; not entered: +inf.  The
        // decode and the slab run x and y in packed FP32 (each lane of
        // v_pk_mul_f32 / v_pk_add_f32 rounds as the scalar operation does)
        const f2 org = {R0.x, R0.y}, sxy = {sx, sy}, oxy = {o.x, o.y}, ixy = {inv.x, inv.y};
        float k[4];
        int ks[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int sh = 8 * i;
            const f2 lxy = org + f2{(float)((qlx >> sh) & 0xFFu), (float)((qly >> sh) & 0xFFu)} * sxy;
            const f2 hxy = org + f2{(float)((qhx >> sh) & 0xFFu), (float)((qhy >> sh) & 0xFFu)} * sxy;
            const float lz = R0.z + (float)((qlz >> sh) & 0xFFu) * sz, hz = R0.z + (float)((qhz >> sh) & 0xFFu) * sz;
            const f2 t0 = (lxy - oxy) * ixy, t1 = (hxy - oxy) * ixy;
            const float t0z = (lz - o.z) * inv.z, t1z = (hz - o.z) * inv.z;
            const float te = fmaxf(fmaxf(fminf(t0.x, t1.x), fminf(t0.y, t1.y)), fminf(t0z, t1z));
            const float tx = fminf(fminf(fmaxf(t0.x, t1.x), fmaxf(t0.y, t1.y)), fmaxf(t0z, t1z));
            const bool ind = tx > te && tx > kTMin;
            const uint32_t f = (fl >> sh) & 0xFFu;
            const float rf = (f & 2u) ? __builtin_inff() : ((f & 4u) ? nr : kRelax);
            k[i] = (i < n && ind && accel_enter_r(te, closest, rf)) ? te : __builtin_inff();
            ks[i] = i;
        }
        // sort by (t_enter, slot): a five-comparator network; every key is
        // distinct in slot, so the order is the model's insertion order
#define RT_WCE(a, b)                                                                       \
        {                                                                                  \
            const bool sw = k[a] > k[b] || (k[a] == k[b] && ks[a] > ks[b]);                \
            const float tk = sw ? k[b] : k[a];                                             \
            k[b] = sw ? k[a] : k[b];                                                       \
            k[a] = tk;                                                                     \
            const int ts = sw ? ks[b] : ks[a];                                             \
            ks[b] = sw ? ks[a] : ks[b];                                                    \
            ks[a] = ts;                                                                    \
        }
        RT_WCE(0, 1) RT_WCE(2, 3) RT_WCE(0, 2) RT_WCE(1, 3) RT_WCE(1, 2)
#undef RT_WCE
        const int h = (k[0] != __builtin_inff()) + (k[1] != __builtin_inff()) + (k[2] != __builtin_inff()) +
                      (k[3] != __builtin_inff());
        if (h > 0) {
            if (sp + h - 1 > kWideStackK) {
                ovf = true;
                return false;
            }
            const auto link = [&](int slot) -> uint32_t {
                const uint32_t f = (fl >> (8 * slot)) & 0xFFu;
                return (base + (uint32_t)slot) | ((f & 1u) << 31) | ((f & 2u) << 29) | ((f & 4u) << 27);
            };
#pragma unroll
            for (int j = 3; j >= 1; --j) {
                if (j < h) {
                    sl[sp * 64 + lane] = link(ks[j]);
                    st[sp * 64 + lane] = (unsigned short)(__float_as_uint(k[j]) >> 16);
                    ++sp;
                }
            }
            cur = link(ks[0]);
            pop = false;
        }
    }
    if (pop) {
        const float thr = closest * kRelax + kRelaxAbs;
        for (;;) {
            if (sp == 0) return false;
            --sp;
            const uint32_t l = sl[sp * 64 + lane];
            if ((l & (kWThin | kWWider)) || __uint_as_float((uint32_t)st[sp * 64 + lane] << 16) <= thr) {
                cur = l;
                break;
            }
        }
    }
    return true;
}

// ------------------------------------------------------------ frontier walk --
//
// The whole wave walks ONE ray (arguments wave-uniform), like coop_walk, but
// each round trip expands up to 64 subtrees of a preorder-sorted frontier
// instead of a contiguous window, so a round follows the walk down every live
// branch at once (a heavy segment takes ~17 rounds, about the tree depth,
// against ~50 windows; tools/frontier_model.py).
//
// The frontier F (per-wave LDS stack, front = top) holds, in preorder, the
// roots of the disjoint subtrees still to finish, some already tested:
//   x = node | L(node) << 31, y = skip(node) (a tested leaf: its triangle),
//   z = t_enter of the node's box (it hit at the closest_t of its insertion),
//   w = kUnres, or 0 (internal: its live children follow it in F), or the
//       leaf's triangle t (+inf: no valid intersection).
// Each round:
//   1. replay: entries are finalized from the front in preorder with the exact
//      closest_t, as the reference visits them.  A box that misses now skips
//      the entries of its subtree (node < skip); a tested leaf that hits and
//      improves sets closest_t / hit; counts are node_step's (2 per hit
//      internal node, 1 per hit leaf).  Stops at the first untested entry
//      that still hits;
//   2. expand: up to 64 untested entries that still hit, one per lane: an
//      internal node loads its child-pair record and keeps the children whose
//      boxes hit at this closest_t, a leaf loads its triangle and tests it up
//      to "t < closest_t" (the compare itself is left to the replay).
// closest_t only shrinks, so a box or triangle that misses at an earlier
// closest_t misses at every later one: speculation can only add work, never
// change a result.  When F is empty the walk continues along the skip chain
// of the last finished subtree (the reference's stack below its position).
// If the front cannot be expanded for lack of room (never seen: the cap is
// 4x the reference's 64-entry stack), the walk stops with pos = the
// reference's next node, to be finished by node_step.
constexpr int kFCap = 256;                   // frontier entries per wave (16 B each)
constexpr int kFReserve = 80;                // slots speculation leaves to the front (> 64-deep descent)
constexpr uint32_t kUnres = 0xFFFFFFFFu;

template <bool COUNT>
__device__ __forceinline__ bool frontier_walk(const float4* __restrict__ nodes, const float4* __restrict__ leafs,
                                              const float4* __restrict__ pairs, int end, int& pos, bool& pos_leaf,
                                              V3 o, V3 d, V3 inv, float& closest, int& hit,
                                              unsigned long long& c_node, unsigned long long& c_tri, uint4* F,
                                              int& rounds) {
    const int lane = threadIdx.x & 63;
    int c = pos;          // next chain node (wave-uniform)
    int top = 0;          // entries in F
    int drop = -1;        // entries with node < drop lie in a subtree whose box missed
    // Every iteration finalizes or expands the front; the bound only guards
    // the GPU against a logic error (parity tests would then fail, not hang).
    for (int guard = 0; guard < (1 << 24); ++guard) {
        if (top == 0) {
            if (c >= end) break;
            rounds += 1 << 16;                                   // chain rounds counted apart (diag)
            const float4 A = nodes[2 * c];
            const float4 B = nodes[2 * c + 1];
            float te;
            bool ind;
            slab(A, B, o, inv, te, ind);
            const int sk = (int)(__float_as_uint(A.w) & kIdx);
            if (ind && te < closest) {
                if (lane == 0)
                    F[0] = make_uint4((uint32_t)c | ((__float_as_uint(B.w) & 2u) << 30), (uint32_t)sk,
                                      __float_as_uint(te), kUnres);
                top = 1;
            }
            c = sk;
            continue;
        }
        const int nl = min(top, 64);
        const bool in = lane < nl;
        uint4 e = make_uint4(0u, 0u, 0x7F800000u, 0u);
        if (in) e = F[top - 1 - lane];
        const int node = (int)(e.x & kIdx);
        const bool lf = (e.x >> 31) != 0u;
        const bool unres = in && e.w == kUnres;
        const float te = __uint_as_float(e.z);
        const float tt = __uint_as_float(e.w);
        // 1. replay, vectorised: between two improving hits closest_t is
        // fixed, so every loaded entry's outcome is a lane-local compare; an
        // expanded internal node whose box misses drops the entries of its
        // subtree (node < its skip: a prefix max over the lanes before it).
        // One pass per improving triangle hit.
        bool miss_int = false;       // expanded internal node whose box missed when finalized
        int base = 0, k, cover;
        for (;;) {
            const bool act = in && lane >= base;
            const bool h = te < closest;
            if (act) miss_int = !unres && !lf && !h;
            cover = wave_excl_max(miss_int ? (int)e.y : -1);
            const bool live = act && node >= max(drop, cover);
            const uint64_t stop = __ballot(live && unres && h);
            const int sidx = stop ? __ffsll((long long)stop) - 1 : nl;
            const uint64_t tm = __ballot(live && lf && !unres && h && tt < closest) & lanes_lt(sidx);
            const int f = tm ? __ffsll((long long)tm) - 1 : sidx;
            if (COUNT) {
                const uint64_t r = lanes_lt(f);
                c_node += 2ull * (unsigned long long)__popcll(__ballot(live && !unres && !lf && h) & r);
                c_tri += (unsigned long long)__popcll(__ballot(live && lf && !unres && h) & r);
            }
            if (!tm) {
                k = sidx;
                if (k == nl) drop = max(drop, lane_i(max(cover, miss_int ? (int)e.y : -1), nl - 1));
                break;
            }
            if (COUNT) ++c_tri;                                  // the improving triangle
            closest = lane_f(tt, f);
            hit = lane_i((int)e.y, f);
            base = f + 1;
        }
        top -= k;
        if (k == nl) continue;
        ++rounds;
        // 2. expand (lanes k.. are the region [top - (nl - k), top) of F)
        const int room = kFCap - top;
        const bool cand = in && lane >= k && unres && node >= max(drop, cover) && te < closest;
        const uint64_t CI = __ballot(cand && !lf);
        if (room < 2 && ((CI >> k) & 1ull)) {                    // no room for the front's children
            pos = lane_i(node, k);
            pos_leaf = false;
            return false;
        }
        // The front always fits (room >= 2); other internal nodes only while
        // kFReserve slots stay free for the front's own descent, so the walk
        // cannot stall on a frontier filled by speculation.
        const bool sel = cand && (lf || lane == k || 2 * (lanes_below(CI) + 1) <= room - kFReserve);
        bool hL = false, hR = false;
        uint4 cL = e, cR = e;
        if (sel) {
            if (lf) {
                const float4 P0 = leafs[3 * node + 0];
                const float4 P1 = leafs[3 * node + 1];
                const float4 P2 = leafs[3 * node + 2];
                float t;
                const bool v = tri_test(P0, P1, P2, o, d, t);
                e.y = __float_as_uint(P0.w);
                e.w = v ? __float_as_uint(t) : 0x7F800000u;
            } else {
                const float4 Q0 = pairs[4 * node + 0];
                const float4 Q1 = pairs[4 * node + 1];
                const float4 Q2 = pairs[4 * node + 2];
                const float4 Q3 = pairs[4 * node + 3];
                float teL, teR;
                bool indL, indR;
                slab(Q0, Q1, o, inv, teL, indL);
                slab(make_float4(Q0.w, Q1.w, Q2.w, 0.f), Q2, o, inv, teR, indR);
                const uint32_t rw = __float_as_uint(Q3.x);
                hL = indL && teL < closest;
                hR = indR && teR < closest;
                cL = make_uint4((uint32_t)(node + 1) | (__float_as_uint(Q3.y) != 0u ? 0x80000000u : 0u), rw & kIdx,
                                __float_as_uint(teL), kUnres);
                cR = make_uint4(rw, e.y, __float_as_uint(teR), kUnres);
                e.w = 0u;
            }
        }
        const bool reg = in && lane >= k;
        const uint64_t RM = __ballot(reg), LM = __ballot(hL), RRM = __ballot(hR);
        const int P = lanes_below(RM) + lanes_below(LM) + lanes_below(RRM);
        const int ntop = top - (nl - k) + __popcll(RM) + __popcll(LM) + __popcll(RRM);
        if (reg) {
            F[ntop - 1 - P] = e;
            if (hL) F[ntop - 2 - P] = cL;
            if (hR) F[ntop - 2 - (hL ? 1 : 0) - P] = cR;
        }
        top = ntop;
    }
    pos = end;
    return true;
}

// ------------------------------------------------------------ simple kernel --

// Diagnostic stamp (diag builds only): global realtime clock (100 MHz) and
// the wave's hardware placement.
__device__ __forceinline__ void diag_stamp(unsigned long long* rec, int which) {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    if ((threadIdx.x & 63) == 0) {
        rec[which] = t;
        if (which == 0) {
            unsigned hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            rec[2] = ((unsigned long long)xcc << 32) | hw;
            rec[3] = ((unsigned long long)(blockIdx.y * gridDim.x + blockIdx.x) << 8) | (threadIdx.x >> 6);
        }
    }
}

// Optional features of trace_simple, compiled in only where a schedule needs
// them so the default inner loop carries no extra work.
// (Bits 1, 2 and 4 belonged to the archived split / tiered / priority
// schedules; the values are kept so kernel names in old profiles still match.)
constexpr int kDiagWords = 8;     // per-wave diag record (rtamd.h rt_diag_copy)
constexpr int kFeatCoopTail = 8;  // finish the last coop_lanes walks of a wave cooperatively
constexpr int kFeatExt = kFeatExtBit;   // non-reference extensions (option "extensions", kExt*)
constexpr int kFeatFrontier = 32; // cooperative tail uses frontier_walk (option coop_walk = 1)

constexpr int kFeatFused = 64;    // heavy tiles in the same launch: workgroups k < 64 * split_n run heavy_pixel
constexpr int kFeatWin32 = 128;   // cooperative windows of 32 slots (option coop_window), else 64
constexpr int kFeatPad = 256;     // the production kernels (cooperative tail, no extensions) on records
                                  //   with pad slots (leaf_align); every other variant always reads pad bits
constexpr int kFeatQ1 = 4096;     // split launch, kernel 1: paths alive at bounce split_bounce go to the
                                  //   launch's ray slots (compacted per wave, no atomics)
constexpr int kFeatQ2 = 8192;     // split launch, kernel 2: the slotted paths from bounce split_bounce,
                                  //   64 per wave in slot order
constexpr int kFeatHalf = 2048;   // option accel_half (with kFeatAccel): 16-B slots, half-precision internal
                                  //   boxes (accel_build.h format 1)
constexpr int kFeatWide = 1024;   // option accel_wide (with kFeatAccel): the 4-wide tree (accel_build.h format 2),
                                  //   children ordered by t_enter, a per-lane LDS stack (wide_step)
constexpr int kFeatAccel = 512;   // option accel: the accel records and rules, packed records, the
                                  //   reference-order fallback
constexpr unsigned kHeavyLaneMark = kLearnHeavyMark;   // rt_internal.h

// One pixel of a heavy tile, the whole wave on it (option heavy_fused, the
// workgroups in front of the tile workgroups of the same launch): every
// segment is walked with frontier_walk from the root; the ray, its
// attenuation and the walk are wave-uniform, so every lane computes the same
// values and lane 0 writes the pixel and the counts.  The arithmetic is the
// lockstep kernel's (slab, tri_test, scatter, sky_color), so pixel and counts
// are identical.  It is a branch of its own at the top of the kernel, so the
// tile path's registers are not live in it and the launch keeps the tile
// path's 73 VGPRs (out of line it would need 119 and spill the arguments).
template <bool COUNT>
__device__ __forceinline__ void heavy_pixel(const TraceArgs& a, int f, int lx, int ly, int lyo, uint4* F) {
    const int lane = threadIdx.x & 63;
    const int end = a.scene.end;
    unsigned long long c_seg = 0, c_node = 0, c_tri = 0, c_mat = 0;
    if (lx < a.tw && ly < a.th && (a.list_stride == 0 || a.band_list[f * a.list_stride + ly / a.band_h] >= 0)) {
        uint32_t seed;
        V3 o, d;
        primary_ray(a, f, a.x0 + lx, frame_row(a, f, ly), seed, o, d);
        V3 att = {1.0f, 1.0f, 1.0f};
        V3 fin = {0.0f, 0.0f, 0.0f};
        int rounds = 0;
        for (int b = 0; b < a.max_bounces; ++b) {
            float closest = kTMax;
            int hit = -1;
            const V3 inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};              // :89
            if (COUNT) {
                ++c_seg;
                if (end > 0) ++c_node;                                       // the root visit
            }
            if (end > 0) {
                int p = 0;
                bool pl = false;
                if (!frontier_walk<COUNT>(a.scene.nodes, a.scene.leafs, a.scene.pairs, end, p, pl, o, d, inv, closest,
                                          hit, c_node, c_tri, F, rounds))
                    while (p < end) p = node_step<COUNT>(a.scene.nodes, a.scene.leafs, p, pl, o, d, inv, closest, hit,
                                                         c_node, c_tri);
            }
            if (hit < 0) {                                                    // :224-226
                fin = vmul(att, sky_color(d));
                break;
            }
            if (COUNT) ++c_mat;
            const V3 hp = vadd(o, vscale(d, closest));                        // ray_at :77-79
            const V3 nrm = hit_normal(a.scene.norms, hit, d);
            const float4 M = a.scene.mats[kShadeStride * hit];
            V3 nd;
            if (!scatter(M, d, nrm, seed, nd)) break;                        // attenuation = 0: black
            att = vmul(att, V3{M.x, M.y, M.z});
            o = hp;
            d = nd;
            // b == max_bounces - 1 leaves fin black (:229-231)
        }
        if (lane == 0) write_pixel(a, lx, lyo, fin);
    }
    if (COUNT) {
        if (lane != 0) c_seg = c_node = c_tri = c_mat = 0;                  // wave-uniform: counted once
        flush_counters(a.counters, c_seg, c_node, c_tri, c_mat);
    }
}

// Occupancy floor for trace_simple (waves per SIMD).  Unconstrained, the
// walk-2 build takes ~70 VGPRs (7 waves).  One frame at a time more waves did
// not pay (round 1); with frames in flight the device is throughput-bound and
// they do: at 7 (round 2, before the compact records) config 3 0.328-0.330 vs
// 0.344-0.346 ms (profiles/r02/occupancy/wpe7); with the compact records, 8
// waves (64 VGPRs, ~20 B per lane of per-segment spills) beat 7 on config 3
// (0.298-0.299 vs 0.301-0.302 ms) and config 6 (0.343-0.344 vs 0.364-0.365),
// config 5 even (profiles/r02/occupancy/wpe8).  The frontier (heavy-tile)
// instantiations keep their registers.
#ifndef RT_SIMPLE_WPE
#define RT_SIMPLE_WPE 8
#endif
// option accel's kernels (A/B builds: make variant FLAGS=-DRT_ACCEL_WPE=7)
#ifndef RT_ACCEL_WPE
#define RT_ACCEL_WPE RT_SIMPLE_WPE
#endif
// 1 = an accel leaf's triangle is loaded only once its box is hit (a second
// dependent round trip for the quarter of leaf visits that test it, two loads
// fewer for the rest); 0 = with the leaf's box, as the reference-order walk
#ifndef RT_ACC_LAZY
#define RT_ACC_LAZY 0
#endif
// s_setprio level of a wave while it walks: the walk's dependent chain
// (record, slab test, next address, next load) issues ahead of the waves that
// shade, whose VALU work is not on any load's path.  1, 2 and 3 measured alike,
// 1.0-1.5% per frame on configs 3 and 5 against 0 (profiles/r06/r6ab, r6ac).
#ifndef RT_WALK_PRIO
#define RT_WALK_PRIO 2
#endif
// 1 = option accel's format-0 walk starts inside the root (DevScene::root_enter;
// A/B builds: 0 = the root's slab test first, as the model's orc_accel_root(0))
#ifndef RT_ROOT_ENTER
#define RT_ROOT_ENTER 1
#endif
template <bool COUNT, bool DIAG = false, int FEAT = 0, int WALK = 2>
__global__ __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu((FEAT & kFeatFrontier) ? 1 : (FEAT & kFeatAccel) ? RT_ACCEL_WPE : RT_SIMPLE_WPE)))
void trace_simple(TraceArgs a) {
    // Pad bits (leaf_align): the production kernels (cooperative tail, no
    // extensions or frontier tail) read them only when built with kFeatPad, so
    // scenes with packed records run the packed code; every other variant
    // reads them always.
    constexpr bool ACC = (FEAT & kFeatAccel) != 0;
    constexpr bool HALF = ACC && (FEAT & kFeatHalf) != 0;
    constexpr bool WIDE = ACC && (FEAT & kFeatWide) != 0;
    constexpr bool PAD = !ACC && ((FEAT & kFeatPad) || (FEAT & (kFeatExt | kFeatFrontier)) || !(FEAT & kFeatCoopTail));
    constexpr bool Q1 = (FEAT & kFeatQ1) != 0, Q2 = (FEAT & kFeatQ2) != 0;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    // frontier_walk's per-wave frontiers (kFCap entries per wave; dynamic LDS,
    // sized by the launch for variants with kFeatFrontier or kFeatFused)
    extern __shared__ uint4 fr[];
    // Split kernel 2: a fixed grid of one-wave workgroups; wave k takes the
    // slotted paths 64k .. 64k + 63 (then 64 (k + grid) ..), in slot order.
    unsigned q_k = Q2 ? blockIdx.x : 0u;
    const unsigned q_total = Q2 ? a.q_prefix[a.q_waves - 1] + a.q_count[a.q_waves - 1] : 0u;
    if (Q2 && q_k * 64u >= q_total) return;
    // One wave = one tile of 64 pixels, (8 << s) x (8 >> s) with s = a.wave_tile
    // (s = 0: 8x8, the reference's local_size 8x8x1, compute_dynamic_ray.comp:157);
    // a workgroup = block_waves (4 or 1) such tiles side by side.
    const int s = a.wave_tile;
    const int tw_w = 8 << s, th_w = 8 >> s;
    // Heavy-first order (option heavy_first): workgroup k takes the k-th most
    // expensive tile of an earlier launch of the same frame, so the frame's
    // longest waves start first.  Only the tile each wave traces changes.
    // With split_n > 0 (the heavy-tile launch) the first split_n tiles of the
    // order are traced one pixel per wave (64 workgroups per tile): the wave's
    // single live lane walks every segment cooperatively (frontier walk).
    int bx = blockIdx.x, by = blockIdx.y, sub = -1;
    unsigned long long skip_lanes = 0;                   // heavy pixels this tile wave leaves out
    // Diagnostic record of this wave and the tile of its per-pixel walk
    // lengths (diag builds): the wave's index in the grid, except in a fused
    // launch in a tile order, where tile t's wave records at n_heavy_px + t and
    // its pixels at t * 64 + lane (a learning launch in another camera's order
    // still gives each tile its own record: rt_learn.hip reads them by tile).
    const int k_wave = (blockIdx.y * gridDim.x + blockIdx.x) * a.block_waves + wave;
    int rec_id = k_wave, tile_id = k_wave, hq = -1;
    if (a.tile_order) {                                  // 1-D grid over the ordered tiles
        const int k = blockIdx.x;
        int t;
        if ((FEAT & kFeatFused) && k < a.n_heavy_px) {   // a heavy pixel (tile * 64 + lane), dispatched first
            hq = a.heavy_px[k];
            t = hq >> 6;
            sub = hq & 63;
        } else if (k < 64 * a.split_n) {
            t = a.tile_order[k >> 6];
            sub = k & 63;
        } else {
            t = a.tile_order[k - 63 * a.split_n - ((FEAT & kFeatFused) ? a.n_heavy_px : 0)];
            if ((FEAT & kFeatFused) && a.tile_mask) skip_lanes = a.tile_mask[t];
            if (FEAT & kFeatFused) {
                rec_id = a.n_heavy_px + t;
                tile_id = t;
            } else if (DIAG && a.diag_lane && a.split_n == 0) {
                // a learning launch in a reused order without heavy pixels (a
                // schedule that does not split them out): records by tile too,
                // as rt_learn.hip reads them
                rec_id = t;
                tile_id = t;
            }
        }
        bx = t % a.tiles_x;
        by = t / a.tiles_x;
    }
    unsigned long long* drec = nullptr;
    if (DIAG) {
        drec = a.diag + kDiagWords * (size_t)rec_id;
        diag_stamp(drec, 0);
    }
    if ((FEAT & kFeatFused) && sub >= 0) {               // a heavy tile's pixel, dispatched first
        const int hf = by / a.tiles_y;                   // its frame of the batch
        const int hy = (by - hf * a.tiles_y) * th_w + (sub >> (3 + s));
        heavy_pixel<COUNT>(a, hf, bx * tw_w + (sub & (tw_w - 1)), hy, (a.row_off ? a.row_off[hf] : hf * a.th) + hy, fr);
        if (DIAG) {
            diag_stamp(drec, 1);
            if (lane == 0) {
                drec[4] = 0;
                drec[5] = 0;
                drec[6] = 0;
                drec[7] = 0;
                // a learning launch: a pixel traced as heavy keeps its place
                // among the heavy ones (its lockstep length is unknown here)
                if (a.diag_lane && hq >= 0) a.diag_lane[hq] = kHeavyLaneMark;
            }
        }
        return;
    }
    const int tl = sub >= 0 ? sub : lane;                // the tile pixel this lane traces
    const int col = bx * a.block_waves + wave;           // wave-tile column
    const int fr_i = by / a.tiles_y;                     // the wave's frame of the batch (tile rows of frame
    by -= fr_i * a.tiles_y;                              //   f follow those of frame f - 1)
    int lx = col * tw_w + (tl & (tw_w - 1));
    const int ly = by * th_w + (tl >> (3 + s));          // row within the frame's rows
    // output row (per-frame offsets: rt_render_batch_runs_device packs each
    // frame's rows after the previous frame's)
    int lyo = (a.row_off ? a.row_off[fr_i] : fr_i * a.th) + ly;
    // (a per-frame band list's -1 entries are padding rows: no pixel)
    const bool pixel = !Q2 && lx < a.tw && ly < a.th && (sub < 0 || lane == 0) && !((skip_lanes >> lane) & 1ull) &&
                       (a.list_stride == 0 || a.band_list[fr_i * a.list_stride + ly / a.band_h] >= 0);
    // Split kernel 1: this wave's slot count starts at 0 (a wave whose paths
    // all end before split_bounce never writes it again)
    if (Q1 && lane == 0) a.q_count[k_wave] = 0u;
    const int coop_lanes = sub >= 0 ? 64 : a.coop_lanes;
    const float4* __restrict__ nodes = a.scene.nodes;
    const float4* __restrict__ leafs = a.scene.leafs;
    const float4* __restrict__ pairs = a.scene.pairs;
    const int end = a.scene.end;                         // node index end (walk 0, the frontier tail)
    const int wend = WALK == 2 ? a.scene.end2 : end;     // the lockstep walk's end: slots for walk 2
    unsigned long long c_seg = 0, c_node = 0, c_tri = 0, c_mat = 0;
    unsigned long long d_iters = 0, d_windows = 0, d_coop_t = 0;   // diag builds only
    unsigned long long d_lane_windows = 0;           // diag: cooperative windows spent on this lane's walks

  do {   // split kernel 2 loops over its packs of 64 slotted paths; every other kernel runs once
    uint32_t seed = 0;
    V3 o = {0.f, 0.f, 0.f}, d = {0.f, 0.f, 1.f};
    V3 att = {1.0f, 1.0f, 1.0f};
    bool alive = pixel;
    int b0 = 0;
    if (Q2) {
        // path i of the slot order: source wave w with prefix[w] <= i < prefix[w + 1]
        const unsigned i = q_k * 64u + (unsigned)lane;
        alive = i < q_total;
        b0 = a.split_bounce;
        if (alive) {
            int lo = 0, hi = a.q_waves;                  // prefix[lo] <= i < prefix[hi] (prefix[q_waves] = total)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (a.q_prefix[mid] <= i) lo = mid;
                else hi = mid;
            }
            const float4* r = a.q_slots + 3 * ((size_t)lo * 64 + (i - a.q_prefix[lo]));
            const float4 r0 = r[0], r1 = r[1], r2 = r[2];
            o = {r0.x, r0.y, r0.z};
            d = {r0.w, r1.x, r1.y};
            att = {r1.z, r1.w, r2.x};
            seed = __float_as_uint(r2.y);
            const int pq = __float_as_int(r2.z);
            lyo = pq / a.tw;
            lx = pq - lyo * a.tw;
        }
    }
    if (pixel) {
        const int x = a.x0 + lx, y = frame_row(a, fr_i, ly);
        if ((FEAT & kFeatExt) && (a.ext & kExtAccumulate)) {
            // extension: a new sample per frame; frame 0 is the reference's seed (:164)
            seed = (uint32_t)(y * a.width + x) + (uint32_t)a.frame_count * (uint32_t)(a.width * a.height);
            primary_ray_seeded(a, fr_i, x, y, seed, o, d);
        } else {
            primary_ray(a, fr_i, x, y, seed, o, d);
        }
    }

    // The bounce loop (:179) is wave-uniform: a lane whose path has ended
    // stays in it with alive = false, so the cooperative tail below can use
    // every lane of the wave.
    for (int b = b0; b < a.max_bounces; ++b) {
        if (__ballot(alive) == 0) break;
        if (Q1 && b == a.split_bounce) {
            // Split kernel 1: the paths still alive leave for this wave's 64
            // ray slots, packed in lane order (no atomics); kernel 2 takes them.
            const uint64_t m = __ballot(alive);
            if (alive) {
                float4* r = a.q_slots + 3 * ((size_t)k_wave * 64 + (size_t)lanes_below(m));
                r[0] = make_float4(o.x, o.y, o.z, d.x);
                r[1] = make_float4(d.y, d.z, att.x, att.y);
                r[2] = make_float4(att.z, __uint_as_float(seed), __int_as_float(lyo * a.tw + lx), 0.0f);
            }
            if (lane == 0) a.q_count[k_wave] = (unsigned)__popcll(m);
            alive = false;
            break;
        }
        float closest = kTMax;
        int hit = -1;
        const V3 inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};              // :89
        // The walk's position: n = the next node the reference would visit
        // (walk 2: its slot in DevScene::walk; walk 0: its node index).
        int n = 0;
        int lend = wend;                  // accel: the end of this ray's layout
        bool incons = false;              // accel: the hit lies before its own box's t_enter
        int oct = 0;                      // accel: the layout this ray walks
        if (ACC && a.scene.n_layouts == 8) {
            oct = (int)((__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 31) << 1) |
                        ((__float_as_uint(d.z) >> 31) << 2)) & a.scene.oct_mask;
            n = oct * a.scene.layout_slots;
            lend = n + a.scene.layout_slots;
        }
        bool nleaf = a.scene.root_leaf != 0;
        bool walking = alive && end > 0;
        // Format 0 (round 6): the walk starts inside the root.  Entering an
        // internal box whose slab test would fail only tests its children,
        // which fail it too (their boxes lie inside), so results are the
        // same, and every segment saves the root's step; the root's two
        // children count as visited, as when the root is entered.
        if (ACC && !HALF && !WIDE && RT_ROOT_ENTER && a.scene.root_enter) {
            n += 1;
            nleaf = ((a.scene.root_first_leaf >> oct) & 1) != 0;
            if (COUNT && alive) c_node += 2;
        }
        // the wide walk (kFeatWide): the record to read next (a child link:
        // index | flags), the lane's stack depth, and an overflowed stack
        uint32_t wcur = a.scene.root_leaf ? kWLeaf : 0u;
        int wsp = 0;
        bool wovf = false;
        if (COUNT && alive) {
            ++c_seg;
            if (end > 0) ++c_node;                                       // the root visit
        }
        {
            // The per-node walk: one dependent load per visit, lanes in lockstep.
            // walk 2, software-pipelined: the next node's box is requested as soon as
            // this node's slab test has chosen it, before this node's triangle
            // test and the loop control, which then overlap the load.
            // walk 2 reads the walk records (DevScene::walk): a leaf's first
            // slot carries its triangle index and v0.x, and the slot after it,
            // Q0 and Q1, the rest of its triangle.
            float4 A, B, Q0, Q1;
            const float4* __restrict__ wr = a.scene.walk;
            // a buffer resource over the records: the next slot's address is one
            // shift of its index (the offset field adds the 16-B halves); the
            // half-format walk uses it whatever RT_CHAIN is
            const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<float4*>(wr), 0,
                WIDE ? (int)((unsigned)(a.scene.end2 + 1) * 64u)
                     : HALF ? (int)((unsigned)(a.scene.end2 + 4) * 16u) : (int)((unsigned)(a.scene.end2 + 2) * 32u),
                0x00020000);
            if (WIDE) {
                // no prefetch: a step reads its record at the top
            } else if (HALF && walking) {
                A = hbuf(wrs, n);
                if (nleaf) {
                    B = hbuf(wrs, n + 1);
                    Q0 = hbuf(wrs, n + 2);
                    Q1 = hbuf(wrs, n + 3);
                }
            } else if (WALK == 2 && walking) {
                A = wr[2 * n];
                B = wr[2 * n + 1];
                if (nleaf) {
                    Q0 = wr[2 * n + 2];
                    Q1 = wr[2 * n + 3];
                }
            }
            float lim = accel_lim(closest);                          // ACC: closest_t's entry bound
            // the walk's dependent chain issues ahead of waves shading (RT_WALK_PRIO)
            if (RT_WALK_PRIO) __builtin_amdgcn_s_setprio(RT_WALK_PRIO);
            // Option accel's format-0 walk tracks its record as a byte offset
            // (slot << 5; the records stay below 2^27 slots, so it and the
            // layout's end fit 32 bits): the next record's address is one
            // select of two values known before the slab test ends, the
            // skip's being its link word << 5 (the shift drops kForce and the
            // L bit), and the slot index is recovered after the loop.
            constexpr bool BYTES = ACC && !HALF && !WIDE && !PAD && WALK == 2 && RT_CHAIN == 2 &&
                                   !RT_ACC_SCALAR && !RT_ACC_LAZY;
            unsigned nb = (unsigned)n << 5;
            const unsigned lend_b = (unsigned)lend << 5;
            while (walking) {
                if (DIAG) ++d_iters;
                if (WIDE) {
                    walking = wide_step<COUNT>(wrs, fr + (size_t)wave * (kWideStackK * 64 * 6 / 16), o, d, inv, closest,
                                               hit, incons, wcur, wsp, wovf, c_node, c_tri);
                    continue;
                }
                if (WALK == 0) {
                    n = node_step<COUNT>(nodes, leafs, n, nleaf, o, d, inv, closest, hit, c_node, c_tri);
                } else if (HALF) {
                    // Format 1: an internal node is its 16-B slot A (half box,
                    // skip | L(first) << 30 | L(skip) << 31); a leaf is A (lo,
                    // triangle | L(next) << 31), B (hi, v0.x), Q0, Q1, exactly as
                    // format 0's.  Only a step with a lane at a leaf loads more
                    // than A.
                    const uint32_t aw = __float_as_uint(A.w);
                    const uint32_t h0 = __float_as_uint(A.x), h1 = __float_as_uint(A.y), h2 = __float_as_uint(A.z);
                    const float4 lo = nleaf ? A : make_float4(half_lo(h0), half_hi(h0), half_lo(h1), 0.f);
                    const float4 hi = nleaf ? B : make_float4(half_hi(h1), half_lo(h2), half_hi(h2), 0.f);
                    float te;
                    bool ind;
                    slab(lo, hi, o, inv, te, ind);
                    const float rf = nleaf ? ((aw & kThinLeaf) ? __builtin_inff() : kRelax) : a.scene.relax_half;
                    const bool hb = ind && accel_enter_r(te, closest, rf);
                    const int nxt = nleaf ? n + 4 : (hb ? n + 1 : (int)(aw & 0x3FFFFFFFu));
                    const bool nl = ((nleaf || !hb) ? (aw >> 31) : (aw >> 30)) & 1u;
                    const float v0x = B.w;                                   // a leaf's v0.x
                    if (COUNT && hb && !nleaf) c_node += 2;
                    A = hbuf(wrs, nxt);                                      // slot end is padding
                    if (hb && nleaf) {                                       // hit_triangle (:196-200)
                        if (COUNT) ++c_tri;
                        float t;
                        if (tri_test(make_float4(v0x, Q0.x, Q0.y, 0.f), make_float4(Q0.z, Q0.w, Q1.x, 0.f),
                                     make_float4(Q1.y, Q1.z, Q1.w, 0.f), o, d, t) &&
                            accel_take(t, (int)(aw & kTri), closest, hit)) {
                            closest = t;
                            hit = (int)(aw & kTri);
                            incons = t < te;
                        }
                    }
                    if (nl && nxt < lend) {
                        B = hbuf(wrs, nxt + 1);
                        Q0 = hbuf(wrs, nxt + 2);
                        Q1 = hbuf(wrs, nxt + 3);
                    }
                    n = nxt;
                    nleaf = nl;
                } else {
                    float te;
                    bool ind;
                    slab(A, B, o, inv, te, ind);
                    const uint32_t aw = __float_as_uint(A.w), bw = __float_as_uint(B.w);
                    const bool hb = ind && (ACC ? accel_enter_lim(te, lim, aw) : te < closest);
                    // a leaf's next node is its successor, two slots on, whether it
                    // is hit or not (its skip); an internal node's left child is
                    // the next slot (one more past a pad slot: leaf bit 29 of word
                    // [0].w, internal bit 2 of word [1].w)
                    // Packed records (no kFeatPad) take the plain ternary; with pad
                    // bits the selects are written by masks: as ternaries the
                    // compiler branched there, on the dependent chain to the next
                    // load (+7% per frame, profiles/r04/r4j-r4k).
                    int nxt;
                    if (PAD) {
                        const int n_leaf = n + 2 + (int)((aw >> 29) & 1u);
                        const int n_hit = n + 1 + (int)((bw >> 2) & 1u);
                        const int m_hit = -(int)hb, m_leaf = -(int)nleaf;
                        const int n_int = (n_hit & m_hit) | ((int)(aw & kIdx) & ~m_hit);
                        nxt = (n_leaf & m_leaf) | (n_int & ~m_leaf);
                    } else {
#if RT_CHAIN == 1 || RT_CHAIN == 2
                        if (BYTES) {
                            const unsigned tb = nb + (nleaf ? 64u : 32u);    // known before the slab test ends
                            nb = (hb || nleaf) ? tb : (aw << 5);
                            nxt = 0;                                         // (the slot: nb >> 5)
                        } else {
                            const int t = n + 1 + (int)nleaf;                // known before the slab test ends
                            nxt = (hb || nleaf) ? t : (int)(aw & kIdx);
                        }
#else
                        nxt = nleaf ? n + 2 : (hb ? n + 1 : (int)(aw & kIdx));
#endif
                    }
                    // accel records: L(first) is bit 31 of word 7, L(skip) / L(next) bit 31
                    // of word 3 (two sign tests); the reference's: bit 0 of word 7
                    const bool nl = ACC ? ((hb && !nleaf) ? (int)bw < 0 : (int)aw < 0)
                                        : ((((hb && !nleaf) ? bw : (aw >> 31)) & 1u) != 0u);
                    const float v0x = B.w;                                   // a leaf's v0.x
                    if (COUNT && hb && !nleaf) c_node += 2;
#if RT_ACC_SCALAR
                    // one slot for every walking lane: the scalar cache
                    const int nf = __builtin_amdgcn_readfirstlane(nxt);
                    const bool uni = ACC && !PAD && __ballot(nxt != nf) == 0;
                    if (uni) {
                        A = sbuf(wr, 2 * nf);
                        B = sbuf(wr, 2 * nf + 1);
                    } else {
                        A = wbuf(wrs, nxt, 0);                               // slot end is padding
                        B = wbuf(wrs, nxt, 16);
                    }
#elif RT_CHAIN >= 2
                    if (BYTES) {
                        A = wbuf_b(wrs, nb, 0);                              // slot end is padding
                        B = wbuf_b(wrs, nb, 16);
                    } else {
                        A = wbuf(wrs, nxt, 0);                               // slot end is padding
                        B = wbuf(wrs, nxt, 16);
                    }
#elif RT_CHAIN == 1
                    {
                        const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(wr) +
                                                                          ((size_t)(unsigned)nxt << 5));
                        A = p[0];                                            // slot end is padding
                        B = p[1];
                    }
#else
                    A = wr[2 * nxt];                                         // slot end is padding
                    B = wr[2 * nxt + 1];
#endif
                    if (hb && nleaf) {                                       // hit_triangle (:196-200)
                        if (COUNT) ++c_tri;
#if RT_CHAIN >= 2
                        if (ACC && RT_ACC_LAZY) {
                            Q0 = wbuf(wrs, n, 32);
                            Q1 = wbuf(wrs, n, 48);
                        }
#endif
                        float t;
                        if (tri_test(make_float4(v0x, Q0.x, Q0.y, 0.f), make_float4(Q0.z, Q0.w, Q1.x, 0.f),
                                     make_float4(Q1.y, Q1.z, Q1.w, 0.f), o, d, t) &&
                            (ACC ? accel_take(t, (int)(aw & kTri), closest, hit) : t < closest)) {
                            closest = t;
                            hit = (int)(aw & kTri);
                            if (ACC) {
                                incons = t < te;
                                lim = accel_lim(t);
                            }
                        }
                    }
                    const bool inb = BYTES ? nb < lend_b : nxt < (ACC ? lend : wend);
                    if (nl && inb && !(ACC && RT_ACC_LAZY)) {
#if RT_ACC_SCALAR
                        if (uni) {
                            Q0 = sbuf(wr, 2 * nf + 2);
                            Q1 = sbuf(wr, 2 * nf + 3);
                        } else {
                            Q0 = wbuf(wrs, nxt, 32);
                            Q1 = wbuf(wrs, nxt, 48);
                        }
#elif RT_CHAIN >= 2
                        if (BYTES) {
                            Q0 = wbuf_b(wrs, nb, 32);
                            Q1 = wbuf_b(wrs, nb, 48);
                        } else {
                            Q0 = wbuf(wrs, nxt, 32);
                            Q1 = wbuf(wrs, nxt, 48);
                        }
#else
                        Q0 = wr[2 * nxt + 2];
                        Q1 = wr[2 * nxt + 3];
#endif
                    }
                    if (!BYTES) n = nxt;
                    nleaf = nl;
                    walking = inb;
                }
                if (WALK == 0 || HALF) walking = n < (ACC ? lend : wend);
                if ((FEAT & kFeatCoopTail) && __popcll(__ballot(walking)) <= coop_lanes) break;
            }
            if (BYTES) n = (int)(nb >> 5);
            if (RT_WALK_PRIO) __builtin_amdgcn_s_setprio(0);
        }
        if (FEAT & kFeatCoopTail) {
            // Every lane is here.  Finish the remaining walks one ray at a
            // time with the whole wave, each from its next node n.
            uint64_t rem = __ballot(walking);
            unsigned long long tc0 = 0;
            if (DIAG && rem != 0) tc0 = wall_clock64();
            while (rem != 0) {
                const int L = __ffsll((long long)rem) - 1;
                rem &= rem - 1;
                const V3 bo = {lane_f(o.x, L), lane_f(o.y, L), lane_f(o.z, L)};
                const V3 bd = {lane_f(d.x, L), lane_f(d.y, L), lane_f(d.z, L)};
                const V3 bi = {lane_f(inv.x, L), lane_f(inv.y, L), lane_f(inv.z, L)};
                float bc = lane_f(closest, L);
                int bh = lane_i(hit, L);
                bool bx = ACC && lane_i((int)incons, L) != 0;
                unsigned long long cn = 0, ct = 0;   // wave-uniform: counted once, by lane L
                const int start = n;
                int nw = 0;
                if ((FEAT & kFeatFrontier) && a.coop_walk) {
                    // the frontier walk takes node indices: walk 2's slot -> node
                    int p = WALK == 2 ? a.scene.slot_node[lane_i(start, L)] : lane_i(start, L);
                    bool pl = false;
                    if (!frontier_walk<COUNT>(nodes, leafs, pairs, end, p, pl, bo, bd, bi, bc, bh, cn, ct,
                                              fr + wave * kFCap, nw))
                        while (p < end) p = node_step<COUNT>(nodes, leafs, p, pl, bo, bd, bi, bc, bh, cn, ct);
                } else {
                    // the windows walk slots of the walk-2 records (walk 0 hands over a
                    // node index: its slot first)
                    const int ws = WALK == 2 ? lane_i(start, L) : a.scene.node_slot[lane_i(start, L)];
                    nw = coop_walk<COUNT, (FEAT & kFeatWin32) ? 32 : 64, PAD, ACC>(
                        a.scene.walk, ACC ? lane_i(lend, L) : a.scene.end2, ws, bo, bd, bi, bc, bh, cn, ct, bx);
                }
                if (DIAG) {
                    d_windows += nw;
                    if (lane == L) d_lane_windows += nw;
                }
                if (lane == L) {
                    closest = bc;
                    hit = bh;
                    if (ACC) incons = bx;
                    if (COUNT) {
                        c_node += cn;
                        c_tri += ct;
                    }
                }
            }
            if (DIAG && tc0) d_coop_t += wall_clock64() - tc0;
        }
        if (ACC) {
            // The fallback: a hit before its own box's t_enter
            // is the one case where the reference's result depends on its
            // visit order; such a segment is walked again, in the reference's
            // order over the reference's records, by the whole wave.
            uint64_t redo = __ballot(alive && ((hit >= 0 && incons) || (WIDE && wovf)));
            while (redo != 0) {
                const int L = __ffsll((long long)redo) - 1;
                redo &= redo - 1;
                const V3 bo = {lane_f(o.x, L), lane_f(o.y, L), lane_f(o.z, L)};
                const V3 bd = {lane_f(d.x, L), lane_f(d.y, L), lane_f(d.z, L)};
                const V3 bi = {lane_f(inv.x, L), lane_f(inv.y, L), lane_f(inv.z, L)};
                float bc = kTMax;
                int bh = -1;
                bool bx = false;
                unsigned long long cn = 1, ct = 0;   // the reference walk's root visit
                coop_walk<COUNT, (FEAT & kFeatWin32) ? 32 : 64, true, false>(a.scene.walk_ref, a.scene.end2_ref, 0,
                                                                             bo, bd, bi, bc, bh, cn, ct, bx);
                if (lane == L) {
                    closest = bc;
                    hit = bh;
                    if (COUNT) {
                        c_node += cn;
                        c_tri += ct;
                    }
                }
            }
        }
        if ((FEAT & kFeatExt) && alive && a.scene.n_spheres > 0)
            sphere_tests(a.scene.spheres, a.scene.n_spheres, o, d, closest, hit);   // extension: spheres
        if (alive) {
            // A path that ends here writes its pixel now, so its final colour
            // is not carried (in registers) through the remaining bounces.
            V3 fin = {0.0f, 0.0f, 0.0f};
            if ((FEAT & kFeatExt) ? hit != -1 : hit >= 0) {               // :212
                if (COUNT) ++c_mat;
                const V3 hp = vadd(o, vscale(d, closest));                  // ray_at :77-79
                V3 nrm;
                float4 M;
                if ((FEAT & kFeatExt) && hit < -1) {                      // extension: a sphere
                    nrm = sphere_normal(a.scene.spheres[2 * (-2 - hit)], hp, d);
                    M = a.scene.spheres[2 * (-2 - hit) + 1];
                } else {
                    nrm = hit_normal(a.scene.norms, hit, d);
                    M = a.scene.mats[kShadeStride * hit];
                }
                V3 nd;
                if ((FEAT & kFeatExt) && (a.ext & kExtEmissive) && M.w == 3.0f) {
                    fin = vmul(att, V3{M.x, M.y, M.z});                   // extension: type 3 emits
                    alive = false;
                } else if (!scatter(M, d, nrm, seed, nd)) {
                    alive = false;                                        // attenuation = 0: black
                } else {
                    att = vmul(att, V3{M.x, M.y, M.z});
                    o = hp;
                    d = nd;
                    if (b == a.max_bounces - 1) alive = false;            // :229-231: black
                }
            } else {
                if (!((FEAT & kFeatExt) && (a.ext & kExtSkyToggle) && a.sky_enabled == 0))
                    fin = vmul(att, sky_color(d));                        // (extension: sky off is black)
                alive = false;
            }
            if (!alive) finish_pixel<FEAT>(a, lx, lyo, fin);
        }
    }
    // A path still alive here ran no bounce at all (max_bounces 0): black.
    if (alive) finish_pixel<FEAT>(a, lx, lyo, V3{0.0f, 0.0f, 0.0f});
    q_k += gridDim.x;
  } while (Q2 && q_k * 64u < q_total);
    if (COUNT) flush_counters(a.counters, c_seg, c_node, c_tri, c_mat);
    if (DIAG) {
        diag_stamp(drec, 1);
        // each pixel's own walk length: its lockstep steps (d_iters counts the
        // loop iterations this lane walked) + 2 x the windows spent on it
        // (a lane whose heavy pixel a one-pixel wave traced leaves that wave's mark)
        if (a.diag_lane && !((skip_lanes >> lane) & 1ull))
            a.diag_lane[(size_t)tile_id * 64 + lane] = (unsigned)(d_iters + 2 * d_lane_windows);
        // the lanes' own lockstep steps, summed (the useful lane-steps of
        // the wave's lockstep walk: lane utilisation = sum / (64 x word 4))
        unsigned long long d_sum = d_iters;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            d_sum += __shfl_xor(d_sum, off);
            const unsigned long long o2 = __shfl_xor(d_iters, off);   // the wave's iterations = the longest lane's
            d_iters = o2 > d_iters ? o2 : d_iters;
        }
        if (lane == 0) {
            drec[4] = d_iters;
            drec[5] = d_windows;
            drec[6] = d_coop_t;
            drec[7] = d_sum;
        }
    }
}

}  // namespace

// The fused heavy-pixel launch (walk 2), in the window size and record form
// of the scene (big: kFeatWin32 | kFeatPad).
#define RT_FUSED(G)                                                                                           \
    if (a.diag) hipLaunchKernelGGL((trace_simple<false, true, FF, 2>), G, block, shm, stream, ao);             \
    else if (a.counters) hipLaunchKernelGGL((trace_simple<true, false, FF, 2>), G, block, shm, stream, ao);     \
    else hipLaunchKernelGGL((trace_simple<false, false, FF, 2>), G, block, shm, stream, ao);
#define RT_FUSED_BIG(G)                                                                                       \
    switch (big) {                                                                                            \
        case kFeatWin32: { constexpr int FF = kFeatCoopTail | kFeatFused | kFeatWin32; RT_FUSED(G) } break;   \
        case kFeatPad: { constexpr int FF = kFeatCoopTail | kFeatFused | kFeatPad; RT_FUSED(G) } break;       \
        case kFeatWin32 | kFeatPad: {                                                                         \
            constexpr int FF = kFeatCoopTail | kFeatFused | kFeatWin32 | kFeatPad;                            \
            RT_FUSED(G)                                                                                       \
        } break;                                                                                              \
        default: { constexpr int FF = kFeatCoopTail | kFeatFused; RT_FUSED(G) } break;                        \
    }

hipError_t launch_trace(const TraceArgs& a, hipStream_t stream, int* kernels) {
    if (kernels) *kernels = 1;
    const int tw_w = 8 << a.wave_tile, th_w = 8 >> a.wave_tile, bw = a.block_waves;
    const int tiles_y = (a.th + th_w - 1) / th_w;       // wave-tile rows of one frame
    dim3 grid((a.tw + bw * tw_w - 1) / (bw * tw_w), a.n_frames * tiles_y);
    const dim3 block(64 * bw);
    const int feat = (a.coop_lanes > 0 ? kFeatCoopTail : 0) | (a.ext != 0 ? kFeatExt : 0) |
                     (a.coop_lanes > 0 && a.coop_walk ? kFeatFrontier : 0);
    // the production kernels (walk 2, coop tail, no extensions or frontier
    // tail) come in both window sizes, for packed and for padded records
    const bool prod = a.walk == 2 && (feat & ~kFeatFrontier) == kFeatCoopTail;
    const int big = prod ? ((a.coop_win == 32 ? kFeatWin32 : 0) | (a.scene.padded ? kFeatPad : 0)) : 0;
    TraceArgs ao = a;
    ao.tiles_y = tiles_y;
    bool join = false;
    if (a.scene.n_layouts > 0 && (a.n_heavy_px > 0 || a.heavy_tiles > 0 || a.walk != 2)) {
        set_error("accel launch with heavy tiles / pixels or walk %d", a.walk);   // plan_order never asks for it
        return hipErrorInvalidValue;
    }
    if (a.tile_order) {      // heavy-first: a 1-D grid over the ordered tiles
        ao.tiles_x = (int)grid.x;
        ao.split_n = 0;
        const int n_tiles = (int)(grid.x * grid.y);
        const int H = std::min(a.heavy_tiles, n_tiles - 1);
        if (a.n_heavy_px > 0 && a.heavy_fused && bw == 1 && (feat & ~kFeatFrontier) == kFeatCoopTail) {
            // One launch: the heavy pixels' one-pixel workgroups first, then
            // every tile without its heavy pixels.
            ao.split_n = 0;
            const dim3 gf(a.n_heavy_px + n_tiles);
            const size_t shm = kFCap * sizeof(uint4);
            RT_FUSED_BIG(gf)
            return hipGetLastError();
        }
        if (H > 0 && a.heavy_fused && bw == 1 && (feat & ~kFeatFrontier) == kFeatCoopTail) {
            // One launch: the H heaviest tiles' one-pixel workgroups first
            // (dispatched in index order, so they start at once), then the
            // other tiles.
            ao.split_n = H;
            const dim3 gf(64 * H + (n_tiles - H));
            const size_t shm = kFCap * sizeof(uint4);
            RT_FUSED_BIG(gf)
            return hipGetLastError();
        }
        if (H > 0 && a.ev_fork && bw == 1 && (feat & ~kFeatFrontier) == kFeatCoopTail) {
            // The H most expensive tiles, one pixel per wave, every segment
            // walked cooperatively with the frontier walk, on an auxiliary
            // stream concurrent with the other tiles' launch.
            const hipStream_t hs = a.aux_stream ? a.aux_stream : stream;   // null: same stream, in sequence
            hipError_t e = hipSuccess;
            if (a.aux_stream) {
                e = hipEventRecord(a.ev_fork, stream);
                if (e == hipSuccess) e = hipStreamWaitEvent(a.aux_stream, a.ev_fork, 0);
                if (e != hipSuccess) return e;
            }
            TraceArgs ah = ao;
            ah.split_n = H;
            ah.coop_walk = 1;
            const dim3 gh(64 * H);
            const size_t shm = kFCap * sizeof(uint4);
            constexpr int FH = kFeatCoopTail | kFeatFrontier;
            if (a.diag) hipLaunchKernelGGL((trace_simple<false, true, FH, 2>), gh, block, shm, hs, ah);
            else if (a.counters) hipLaunchKernelGGL((trace_simple<true, false, FH, 2>), gh, block, shm, hs, ah);
            else hipLaunchKernelGGL((trace_simple<false, false, FH, 2>), gh, block, shm, hs, ah);
            e = hipGetLastError();
            if (e == hipSuccess && a.aux_stream) e = hipEventRecord(a.ev_join, a.aux_stream);
            if (e != hipSuccess) return e;
            if (kernels) *kernels = 2;
            ao.tile_order = a.tile_order + H;
            if (a.diag) ao.diag = a.diag + (size_t)kDiagWords * gh.x;
            grid = dim3(n_tiles - H);
            join = a.aux_stream != nullptr;
        } else {
            grid = dim3(n_tiles);
        }
    }
    const size_t shm_f = (size_t)bw * kFCap * sizeof(uint4);   // kFeatFrontier variants only
    const size_t shm_w = (size_t)bw * kWideStackK * 64 * 6;       // kFeatWide: the lanes' stacks
#define RT_SHM(F) (((F) & kFeatFrontier) ? shm_f : ((F) & kFeatWide) ? shm_w : 0)
#define RT_SIMPLE(F, W)                                                                                         \
    if (a.diag) hipLaunchKernelGGL((trace_simple<false, true, F, W>), grid, block, RT_SHM(F), stream, ao);           \
    else if (a.counters) hipLaunchKernelGGL((trace_simple<true, false, F, W>), grid, block, RT_SHM(F), stream, ao); \
    else hipLaunchKernelGGL((trace_simple<false, false, F, W>), grid, block, RT_SHM(F), stream, ao);
    if (a.scene.n_layouts > 0) {
        // option accel (walk 2 records; the launcher never splits heavy tiles
        // or pixels out of an accel launch, and there is no frontier tail)
        if (a.q_slots && a.split_bounce > 0 && a.split_bounce < a.max_bounces && feat == 0 && !a.scene.half &&
            !a.scene.wide &&
            !a.diag && !a.counters && (int)(grid.x * grid.y) * bw <= a.q_waves) {
            // split launch: kernel 1 to bounce split_bounce,
            // the scan of its per-wave counts, kernel 2 for the rest
            ao.q_waves = (int)(grid.x * grid.y) * bw;
            hipLaunchKernelGGL((trace_simple<false, false, kFeatAccel | kFeatQ1, 2>), grid, block, 0, stream, ao);
            size_t tb = a.q_temp_bytes;
            const hipError_t se = rocprim::exclusive_scan(a.q_temp, tb, a.q_count, a.q_prefix, 0u,
                                                          (size_t)ao.q_waves, rocprim::plus<unsigned>(), stream);
            if (se != hipSuccess) return se;
            TraceArgs a2 = ao;
            a2.tile_order = nullptr;
            a2.split_n = 0;
            a2.block_waves = 1;
            hipLaunchKernelGGL((trace_simple<false, false, kFeatAccel | kFeatQ2, 2>), dim3(a.q_grid), dim3(64), 0,
                               stream, a2);
            if (kernels) *kernels = 2;                          // the frame kernels (q_scan aside)
            return hipGetLastError();
        }
        if (a.scene.wide) {
            // format 2 records: no cooperative tail (set_schedule: coop_lanes 0)
            if (feat & kFeatCoopTail) {
                set_error("accel_wide launch with coop_lanes %d", a.coop_lanes);
                return hipErrorInvalidValue;
            }
            if (feat & kFeatExt) RT_SIMPLE(kFeatExt | kFeatAccel | kFeatWide, 2)
            else RT_SIMPLE(kFeatAccel | kFeatWide, 2)
            return hipGetLastError();
        }
        if (a.scene.half) {
            // format 1 records: no cooperative tail (set_schedule: coop_lanes 0)
            if (feat & kFeatCoopTail) {
                set_error("accel_half launch with coop_lanes %d", a.coop_lanes);
                return hipErrorInvalidValue;
            }
            if (feat & kFeatExt) RT_SIMPLE(kFeatExt | kFeatAccel | kFeatHalf, 2)
            else RT_SIMPLE(kFeatAccel | kFeatHalf, 2)
            return hipGetLastError();
        }
        switch (feat & ~kFeatFrontier) {
            case kFeatCoopTail:
                if (a.coop_win == 32) RT_SIMPLE(kFeatCoopTail | kFeatAccel | kFeatWin32, 2)
                else RT_SIMPLE(kFeatCoopTail | kFeatAccel, 2)
                break;
            case 0: RT_SIMPLE(kFeatAccel, 2) break;
            default: RT_SIMPLE(kFeatCoopTail | kFeatExt | kFeatAccel, 2) break;
        }
    } else if (a.walk == 2) {
        switch (feat) {
            case kFeatCoopTail:
                switch (big) {
                    case kFeatWin32: RT_SIMPLE(kFeatCoopTail | kFeatWin32, 2) break;
                    case kFeatPad: RT_SIMPLE(kFeatCoopTail | kFeatPad, 2) break;
                    case kFeatWin32 | kFeatPad: RT_SIMPLE(kFeatCoopTail | kFeatWin32 | kFeatPad, 2) break;
                    default: RT_SIMPLE(kFeatCoopTail, 2) break;
                }
                break;
            case 0: RT_SIMPLE(0, 2) break;
            default: RT_SIMPLE(kFeatCoopTail | kFeatExt | kFeatFrontier, 2) break;
        }
    } else {
        switch (feat) {
            case 0: RT_SIMPLE(0, 0) break;
            case kFeatCoopTail: RT_SIMPLE(kFeatCoopTail, 0) break;
            default: RT_SIMPLE(kFeatCoopTail | kFeatExt | kFeatFrontier, 0) break;
        }
    }
#undef RT_SIMPLE
#undef RT_SHM
#undef RT_FUSED_BIG
#undef RT_FUSED
    if (join) {
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, a.ev_join, 0);
        return e;
    }
    return hipGetLastError();
}

}  // namespace rtamd
