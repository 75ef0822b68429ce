// rt_trace.hip — gfx950 path-trace kernels for the reference's per-pixel
// render path (shaders/compute_dynamic_ray.comp, dispatched by
// VulkanEngine.recordComputeCommands, VulkanEngine.java:437-515).
//
// Arithmetic contract: every float operation the shader performs is done here
// in IEEE binary32, in the shader's evaluation order, with no contraction
// (built with -ffp-contract=off) and hipcc's correctly rounded f32 division
// and sqrt.  The CPU oracle (oracle/rt_oracle.c) states the same contract, so
// the two agree bit for bit; see DESIGN.md §Parity.
//
// Traversal: stackless preorder walk over the compact 32-B nodes
// (rt_internal.h), which replays the reference's stack DFS
// (compute_dynamic_ray.comp:185-210) node for node: next = hit ? i+1 : skip(i).
//
// Two schedules of the same per-pixel work:
//   trace_simple      one lane = one pixel for its whole path (the
//                     reference's dispatch shape, 8x8 pixels per wave).
//   trace_persistent  persistent waves; a lane whose path ends pulls the next
//                     pixel from a global queue of 8x8 tiles, and the shading
//                     block (scatter / sky / pixel write) runs only once enough
//                     lanes of the wave have finished a segment, so traversal
//                     steps run with most lanes busy.  Results are identical:
//                     every pixel's path is independent (its RNG seed is its
//                     pixel index, :164) and is computed with the same ops.
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

// Frame row of local row ly (rt_internal.h, TraceArgs band mapping).
__device__ __forceinline__ int frame_row(const TraceArgs& a, int ly) {
    return a.y0 + ((ly / a.band_h) * a.band_stride + a.band_off) * a.band_h + ly % a.band_h;
}

// Seed, AA jitter and primary ray (:164-173).
__device__ __forceinline__ void primary_ray(const TraceArgs& a, int x, int y, uint32_t& seed, V3& o, V3& d) {
    seed = (uint32_t)(y * a.width + x);
    const float u = ((float)x + rnd(seed)) / (float)a.width;
    const float v = ((float)(a.height - 1 - y) + rnd(seed)) / (float)a.height;
    const V3 cam_o = {a.cam.ox, a.cam.oy, a.cam.oz};
    const V3 cam_l = {a.cam.lx, a.cam.ly, a.cam.lz};
    const V3 cam_h = {a.cam.hx, a.cam.hy, a.cam.hz};
    const V3 cam_v = {a.cam.vx, a.cam.vy, a.cam.vz};
    o = cam_o;
    d = vnormalize(vsub(vadd(vadd(cam_l, vscale(cam_h, u)), vscale(cam_v, v)), cam_o));
}

// One node of the walk: hit_aabb (:88-103) and, at a leaf whose box is hit,
// hit_triangle (:105-129).  Returns the next node index.
template <bool COUNT>
__device__ __forceinline__ int node_step(const float4* __restrict__ nodes, const float4* __restrict__ tris,
                                         int i, V3 o, V3 d, V3 inv, float& closest, int& hit,
                                         unsigned long long& c_node, unsigned long long& c_tri) {
    const float4 A = nodes[2 * i];
    const float4 B = nodes[2 * i + 1];
    if (COUNT) ++c_node;
    const float t0x = (A.x - o.x) * inv.x, t1x = (B.x - o.x) * inv.x;
    const float t0y = (A.y - o.y) * inv.y, t1y = (B.y - o.y) * inv.y;
    const float t0z = (A.z - o.z) * inv.z, t1z = (B.z - o.z) * inv.z;
    const float te = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tx = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    const bool hb = tx > te && tx > kTMin && te < closest;
    const int leaf = __float_as_int(B.w);
    if (hb && leaf >= 0) {
        if (COUNT) ++c_tri;
        const float4 P0 = tris[3 * leaf + 0];
        const float4 P1 = tris[3 * leaf + 1];
        const float4 P2 = tris[3 * leaf + 2];
        const V3 v0 = {P0.x, P0.y, P0.z};
        const V3 e1 = {P1.x, P1.y, P1.z};
        const V3 e2 = {P2.x, P2.y, P2.z};
        const V3 pv = vcross(d, e2);
        const float det = vdot(e1, pv);
        if (!(det > -0.00001f && det < 0.00001f)) {
            const float inv_det = 1.0f / det;
            const V3 s = vsub(o, v0);
            const float uu = inv_det * vdot(s, pv);
            if (!(uu < 0.0f || uu > 1.0f)) {
                const V3 q = vcross(s, e1);
                const float vv = inv_det * vdot(d, q);
                if (!(vv < 0.0f || (uu + vv) > 1.0f)) {
                    const float t = inv_det * vdot(e2, q);
                    if (t > kTMin && t < closest) {
                        closest = t;
                        hit = leaf;
                    }
                }
            }
        }
    }
    return hb ? i + 1 : __float_as_int(A.w);
}

// The hit normal of :124-125: normalize(cross(e1,e2)) (precomputed per
// triangle, rt_internal.h), flipped to face against d.
__device__ __forceinline__ V3 hit_normal(const float4* __restrict__ tris, int hit, V3 d) {
    V3 n = {tris[3 * hit + 0].w, tris[3 * hit + 1].w, tris[3 * hit + 2].w};
    if (vdot(d, n) > 0.0f) n = {-n.x, -n.y, -n.z};
    return n;
}

// scatter (:132-154).  Returns true and the new direction / albedo on scatter.
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
// them so the default inner loop carries no extra compares.
constexpr int kFeatSpill = 1;   // split schedule: hand paths on after seg_limit segments
constexpr int kFeatHeavy = 2;   // tiered schedule: hand walks on after heavy_budget visits
constexpr int kFeatPrio = 4;    // raise wave priority after prio_after visits

template <bool COUNT, bool DIAG = false, int FEAT = 0>
__global__ __launch_bounds__(256) void trace_simple(TraceArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    unsigned long long* drec = nullptr;
    if (DIAG) {
        drec = a.diag + 4 * (size_t)((blockIdx.y * gridDim.x + blockIdx.x) * 4 + wave);
        diag_stamp(drec, 0);
    }
    // One wave = one tile of 64 pixels, (8 << s) x (8 >> s) with s = a.wave_tile
    // (s = 0: 8x8, the reference's local_size 8x8x1, compute_dynamic_ray.comp:157);
    // a 256-thread block = 4 such tiles side by side.
    const int s = a.wave_tile;
    const int tw_w = 8 << s, th_w = 8 >> s;
    const int lx = (blockIdx.x * 4 + wave) * tw_w + (lane & (tw_w - 1));
    const int ly = blockIdx.y * th_w + (lane >> (3 + s));
    unsigned long long c_seg = 0, c_node = 0, c_tri = 0, c_mat = 0;
    bool spill = false, heavy = false;
    int steps = 0;

    if (lx < a.tw && ly < a.th) {
        const int x = a.x0 + lx;
        const int y = frame_row(a, ly);
        uint32_t seed;
        V3 o, d;
        primary_ray(a, x, y, seed, o, d);
        V3 fin = {0.0f, 0.0f, 0.0f};
        V3 att = {1.0f, 1.0f, 1.0f};
        for (int b = 0; b < a.max_bounces; ++b) {                         // :179
            if ((FEAT & kFeatSpill) && b == a.seg_limit) {               // hand the path on
                spill = true;
                PathState* st = a.spill + atomicAdd(a.spill_count, 1u);
                st->q0 = make_float4(o.x, o.y, o.z, att.x);
                st->q1 = make_float4(d.x, d.y, d.z, att.y);
                st->q2 = make_float4(att.z, __uint_as_float(seed), __int_as_float(b),
                                     __int_as_float(lx | (ly << 16)));
                break;
            }
            if (COUNT) ++c_seg;
            float closest = kTMax;
            int hit = -1;
            const V3 inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};          // :89
            int i = 0;
            while (i < a.scene.end) {
                i = node_step<COUNT>(a.scene.nodes, a.scene.tris, i, o, d, inv, closest, hit, c_node, c_tri);
                // A wave still walking after prio_after steps holds the frame's
                // critical path: let it win instruction arbitration.
                if (FEAT & (kFeatPrio | kFeatHeavy)) ++steps;
                if ((FEAT & kFeatPrio) && steps == a.prio_after) __builtin_amdgcn_s_setprio(3);
                if ((FEAT & kFeatHeavy) && steps >= a.heavy_budget && i < a.scene.end) {   // hand the walk on
                    heavy = true;
                    HeavyRay* hv = a.heavy + atomicAdd(a.heavy_count, 1u);
                    hv->p.q0 = make_float4(o.x, o.y, o.z, att.x);
                    hv->p.q1 = make_float4(d.x, d.y, d.z, att.y);
                    hv->p.q2 = make_float4(att.z, __uint_as_float(seed), __int_as_float(b),
                                           __int_as_float(lx | (ly << 16)));
                    hv->q3 = make_float4(closest, __int_as_float(i), __int_as_float(hit), 0.0f);
                    break;
                }
            }
            if (heavy) break;
            if (hit >= 0) {                                               // :212
                if (COUNT) ++c_mat;
                const V3 n = hit_normal(a.scene.tris, hit, d);
                const V3 hp = vadd(o, vscale(d, closest));                  // ray_at :77-79
                const float4 M = a.scene.mats[hit];
                V3 nd;
                if (!scatter(M, d, n, seed, nd)) break;                   // attenuation = 0: black
                att = vmul(att, V3{M.x, M.y, M.z});
                o = hp;
                d = nd;
            } else {
                fin = vmul(att, sky_color(d));
                break;
            }
            if (b == a.max_bounces - 1) fin = {0.0f, 0.0f, 0.0f};        // :229-231
        }
        if (!spill && !heavy) write_pixel(a, lx, ly, fin);
    }
    if (COUNT) flush_counters(a.counters, c_seg, c_node, c_tri, c_mat);
    if (DIAG) diag_stamp(drec, 1);
}

// -------------------------------------------------------- persistent kernel --

constexpr int kIdle = 0, kTrace = 1, kReady = 2;

template <bool COUNT>
__global__ __launch_bounds__(256) void trace_persistent(TraceArgs a) {
    const int lane = threadIdx.x & 63;
    const int tiles_x = (a.tw + 7) >> 3;
    // Work slots: 8x8 pixel tiles in row-major tile order, or (resume) the
    // paths the simple pass spilled, in spill order.
    const int n_slots = a.resume ? (int)*a.spill_count : tiles_x * ((a.th + 7) >> 3) * 64;
    const float4* __restrict__ nodes = a.scene.nodes;
    const float4* __restrict__ tris = a.scene.tris;
    const int end = a.scene.end;
    const int shade_min = a.shade_min;

    unsigned long long c_seg = 0, c_node = 0, c_tri = 0, c_mat = 0;
    int pool_next = 0, pool_end = 0;     // wave-uniform: this wave's unclaimed slots
    bool exhausted = false;              // wave-uniform: the global queue is empty

    int mode = kIdle;
    int lx = 0, ly = 0, b = 0, node = 0, hit = -1;
    uint32_t seed = 0;
    float closest = kTMax;
    V3 o = {0.f, 0.f, 0.f}, d = {0.f, 0.f, 1.f}, inv = {0.f, 0.f, 1.f}, att = {1.f, 1.f, 1.f};

    for (;;) {
        // ---- refill idle lanes with new pixels (consecutive slots = one 8x8 tile)
        uint64_t idle = __ballot(mode == kIdle);
        while (idle != 0 && !exhausted) {
            if (pool_next >= pool_end) {
                int base = 0;
                if (lane == 0) base = (int)atomicAdd(a.queue, 64u);
                base = __shfl(base, 0);
                if (base >= n_slots) { exhausted = true; break; }
                pool_next = base;
                pool_end = base + 64;
            }
            const int avail = pool_end - pool_next;
            const int rank = lanes_below(idle);
            if (a.resume) {
                if (mode == kIdle && rank < avail && pool_next + rank < n_slots) {
                    const PathState p = a.spill[pool_next + rank];
                    o = {p.q0.x, p.q0.y, p.q0.z};
                    d = {p.q1.x, p.q1.y, p.q1.z};
                    att = {p.q0.w, p.q1.w, p.q2.x};
                    seed = __float_as_uint(p.q2.y);
                    b = __float_as_int(p.q2.z);
                    const int pix = __float_as_int(p.q2.w);
                    lx = pix & 0xFFFF;
                    ly = pix >> 16;
                    inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
                    closest = kTMax;
                    hit = -1;
                    node = 0;
                    mode = end > 0 ? kTrace : kReady;
                    if (COUNT) ++c_seg;
                }
            } else if (mode == kIdle && rank < avail) {
                const int slot = pool_next + rank;
                const int tile = slot >> 6, w = slot & 63;
                lx = (tile % tiles_x) * 8 + (w & 7);
                ly = (tile / tiles_x) * 8 + (w >> 3);
                if (lx < a.tw && ly < a.th) {
                    const int x = a.x0 + lx, y = frame_row(a, ly);
                    primary_ray(a, x, y, seed, o, d);
                    att = {1.0f, 1.0f, 1.0f};
                    b = 0;
                    inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
                    closest = kTMax;
                    hit = -1;
                    node = 0;
                    mode = end > 0 ? kTrace : kReady;
                    if (COUNT) ++c_seg;
                }
            }
            pool_next += min(__popcll(idle), avail);
            idle = __ballot(mode == kIdle);
        }

        // ---- traversal: step until enough lanes wait to be shaded
        for (;;) {
            if (mode == kTrace) {
                node = node_step<COUNT>(nodes, tris, node, o, d, inv, closest, hit, c_node, c_tri);
                if (node >= end) mode = kReady;
            }
            const uint64_t trace = __ballot(mode == kTrace);
            if (trace == 0 || __popcll(__ballot(mode == kReady)) >= shade_min) break;
        }

        // ---- shading: scatter or sky; next segment, or finish the pixel
        if (mode == kReady) {
            bool finish = true;
            V3 fin = {0.0f, 0.0f, 0.0f};
            if (hit >= 0) {
                if (COUNT) ++c_mat;
                const V3 n = hit_normal(tris, hit, d);
                const V3 hp = vadd(o, vscale(d, closest));
                const float4 M = a.scene.mats[hit];
                V3 nd;
                if (scatter(M, d, n, seed, nd) && b < a.max_bounces - 1) {
                    att = vmul(att, V3{M.x, M.y, M.z});
                    o = hp;
                    d = nd;
                    ++b;
                    inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
                    closest = kTMax;
                    hit = -1;
                    node = 0;
                    mode = end > 0 ? kTrace : kReady;
                    finish = false;
                    if (COUNT) ++c_seg;
                }
                // absorbed (:220-222) or scattered on the last bounce (:229-231): black
            } else {
                fin = vmul(att, sky_color(d));
            }
            if (finish) {
                write_pixel(a, lx, ly, fin);
                mode = kIdle;
            }
        }
        if (exhausted && __ballot(mode != kIdle) == 0) break;
    }
    if (COUNT) flush_counters(a.counters, c_seg, c_node, c_tri, c_mat);
}

// ------------------------------------------------------- cooperative kernel --
//
// One wave walks ONE ray.  The walk is the reference's preorder visit sequence
// (compute_dynamic_ray.comp:185-210), replayed exactly:
//   1. lane k loads node n+k of the window [n, n+64) (2 KB, coalesced) and
//      computes its slab test; leaves whose box is hit at the current
//      closest_t also run the triangle test up to (but not including) the
//      "t < closest_t" compare (:105-122);
//   2. ballots turn "box hit at closest_t" (H), "triangle hit that improves
//      closest_t" (T) and "is a leaf" (Lf) into 64-bit masks;
//   3. the scalar unit replays the walk through the window: node k is hit iff
//      bit k of H; next = k+1 on a hit, skip(k) on a miss; a triangle hit
//      updates closest_t / hit and re-ballots H and T (closest_t only shrinks,
//      so a leaf not pre-tested at the old closest_t cannot hit at the new one).
// Box and triangle tests are the same float operations as node_step, so
// closest_t, the hit and the visit / test counts equal the per-lane walk's.

__device__ __forceinline__ int lane_i(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ float lane_f(float v, int k) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

template <bool COUNT>
__device__ __forceinline__ void coop_walk(const float4* __restrict__ nodes, const float4* __restrict__ tris,
                                          int end, int n, V3 o, V3 d, V3 inv, float& closest, int& hit,
                                          unsigned long long& c_node, unsigned long long& c_tri) {
    const int lane = threadIdx.x & 63;
    while (n < end) {
        const int j = n + lane;
        float te = 0.0f, tt = 0.0f;
        int sk = 0, lf = -1;
        bool ind = false, tv = false;
        if (j < end) {
            const float4 A = nodes[2 * j];
            const float4 B = nodes[2 * j + 1];
            const float t0x = (A.x - o.x) * inv.x, t1x = (B.x - o.x) * inv.x;
            const float t0y = (A.y - o.y) * inv.y, t1y = (B.y - o.y) * inv.y;
            const float t0z = (A.z - o.z) * inv.z, t1z = (B.z - o.z) * inv.z;
            te = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
            const float tx = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
            ind = tx > te && tx > kTMin;
            sk = __float_as_int(A.w);
            lf = __float_as_int(B.w);
            if (ind && lf >= 0 && te < closest) {
                const float4 P0 = tris[3 * lf + 0];
                const float4 P1 = tris[3 * lf + 1];
                const float4 P2 = tris[3 * lf + 2];
                const V3 v0 = {P0.x, P0.y, P0.z};
                const V3 e1 = {P1.x, P1.y, P1.z};
                const V3 e2 = {P2.x, P2.y, P2.z};
                const V3 pv = vcross(d, e2);
                const float det = vdot(e1, pv);
                if (!(det > -0.00001f && det < 0.00001f)) {
                    const float inv_det = 1.0f / det;
                    const V3 s = vsub(o, v0);
                    const float uu = inv_det * vdot(s, pv);
                    if (!(uu < 0.0f || uu > 1.0f)) {
                        const V3 q = vcross(s, e1);
                        const float vv = inv_det * vdot(d, q);
                        if (!(vv < 0.0f || (uu + vv) > 1.0f)) {
                            tt = inv_det * vdot(e2, q);
                            tv = tt > kTMin;
                        }
                    }
                }
            }
        }
        uint64_t H = __ballot(ind && te < closest);
        uint64_t T = __ballot(tv && tt < closest);
        const uint64_t Lf = __ballot(lf >= 0);
        const int lim = min(64, end - n);
        int k = 0;
        while (k < lim) {
            if (COUNT) ++c_node;
            if ((H >> k) & 1ull) {
                if ((Lf >> k) & 1ull) {
                    if (COUNT) ++c_tri;
                    if ((T >> k) & 1ull) {
                        closest = lane_f(tt, k);
                        hit = lane_i(lf, k);
                        H = __ballot(ind && te < closest);
                        T = __ballot(tv && tt < closest);
                    }
                }
                ++k;
            } else {
                k = lane_i(sk, k) - n;
            }
        }
        n += k;
    }
}

template <bool COUNT>
__global__ __launch_bounds__(256) void trace_coop(TraceArgs a) {
    const int lane = threadIdx.x & 63;
    const int end = a.scene.end;
    const int n_rays = (int)*a.heavy_count;
    unsigned long long c_seg = 0, c_node = 0, c_tri = 0, c_mat = 0;   // wave-uniform
    for (;;) {
        int r = 0;
        if (lane == 0) r = (int)atomicAdd(a.queue, 1u);
        r = __builtin_amdgcn_readfirstlane(r);
        if (r >= n_rays) break;
        const HeavyRay hv = a.heavy[r];
        V3 o = {hv.p.q0.x, hv.p.q0.y, hv.p.q0.z};
        V3 d = {hv.p.q1.x, hv.p.q1.y, hv.p.q1.z};
        V3 att = {hv.p.q0.w, hv.p.q1.w, hv.p.q2.x};
        uint32_t seed = __float_as_uint(hv.p.q2.y);
        int b = __float_as_int(hv.p.q2.z);
        const int pix = __float_as_int(hv.p.q2.w);
        float closest = hv.q3.x;
        int node = __float_as_int(hv.q3.y);
        int hit = __float_as_int(hv.q3.z);
        V3 fin = {0.0f, 0.0f, 0.0f};
        for (;;) {
            const V3 inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
            coop_walk<COUNT>(a.scene.nodes, a.scene.tris, end, node, o, d, inv, closest, hit, c_node, c_tri);
            if (hit < 0) {
                fin = vmul(att, sky_color(d));
                break;
            }
            if (COUNT) ++c_mat;
            const V3 n = hit_normal(a.scene.tris, hit, d);
            const V3 hp = vadd(o, vscale(d, closest));
            const float4 M = a.scene.mats[hit];
            V3 nd;
            if (!scatter(M, d, n, seed, nd) || b == a.max_bounces - 1) break;   // black
            att = vmul(att, V3{M.x, M.y, M.z});
            o = hp;
            d = nd;
            ++b;
            closest = kTMax;
            hit = -1;
            node = 0;
            if (COUNT) ++c_seg;
        }
        if (lane == 0) write_pixel(a, pix & 0xFFFF, pix >> 16, fin);
    }
    if (COUNT && lane == 0) {
        atomicAdd(&a.counters->segments, c_seg);
        atomicAdd(&a.counters->node_visits, c_node);
        atomicAdd(&a.counters->tri_tests, c_tri);
        atomicAdd(&a.counters->mat_reads, c_mat);
    }
}

}  // namespace

int persistent_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, trace_persistent<false>, 256, 0) != hipSuccess || n < 1)
        n = 1;
    return n > 8 ? 8 : n;
}

hipError_t launch_trace(const TraceArgs& a, hipStream_t stream) {
    const dim3 block(256);
    if (a.kernel == kKernelTiered) {
        // tier 1: lockstep tiles; paths over the visit budget are suspended
        TraceArgs s = a;
        s.kernel = kKernelSimple;
        hipError_t e = hipMemsetAsync(a.heavy_count, 0, sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
        e = launch_trace(s, stream);
        if (e != hipSuccess) return e;
        // tier 2: one wave per suspended path
        e = hipMemsetAsync(a.queue, 0, sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
        if (a.counters)
            hipLaunchKernelGGL(trace_coop<true>, dim3(a.grid_blocks), block, 0, stream, a);
        else
            hipLaunchKernelGGL(trace_coop<false>, dim3(a.grid_blocks), block, 0, stream, a);
        return hipGetLastError();
    }
    if (a.kernel == kKernelSplit) {
        // pass 1: coherent 8x8 lockstep tiles for the first seg_limit segments
        TraceArgs s = a;
        s.kernel = kKernelSimple;
        s.resume = 0;
        hipError_t e = hipMemsetAsync(a.spill_count, 0, sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
        e = launch_trace(s, stream);
        if (e != hipSuccess) return e;
        // pass 2: the surviving paths, compacted, on persistent waves
        TraceArgs p = a;
        p.kernel = kKernelPersistent;
        p.resume = 1;
        p.seg_limit = 1 << 30;
        return launch_trace(p, stream);
    }
    if (a.kernel == kKernelPersistent) {
        const dim3 grid(a.grid_blocks);
        hipError_t e = hipMemsetAsync(a.queue, 0, sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
        if (a.counters)
            hipLaunchKernelGGL(trace_persistent<true>, grid, block, 0, stream, a);
        else
            hipLaunchKernelGGL(trace_persistent<false>, grid, block, 0, stream, a);
    } else {
        const int tw_w = 8 << a.wave_tile, th_w = 8 >> a.wave_tile;
        const dim3 grid((a.tw + 4 * tw_w - 1) / (4 * tw_w), (a.th + th_w - 1) / th_w);
        const int feat = (a.seg_limit < (1 << 30) ? kFeatSpill : 0) |
                         (a.heavy_budget < (1 << 30) ? kFeatHeavy : 0) | (a.prio_after > 0 ? kFeatPrio : 0);
#define RT_SIMPLE(F)                                                                              \
        if (a.diag) hipLaunchKernelGGL((trace_simple<false, true, F>), grid, block, 0, stream, a); \
        else if (a.counters) hipLaunchKernelGGL((trace_simple<true, false, F>), grid, block, 0, stream, a); \
        else hipLaunchKernelGGL((trace_simple<false, false, F>), grid, block, 0, stream, a);
        switch (feat) {
            case 0: RT_SIMPLE(0) break;
            case kFeatSpill: RT_SIMPLE(kFeatSpill) break;
            case kFeatHeavy: RT_SIMPLE(kFeatHeavy) break;
            case kFeatPrio: RT_SIMPLE(kFeatPrio) break;
            default: RT_SIMPLE(kFeatSpill | kFeatHeavy | kFeatPrio) break;
        }
#undef RT_SIMPLE
    }
    return hipGetLastError();
}

}  // namespace rtamd
