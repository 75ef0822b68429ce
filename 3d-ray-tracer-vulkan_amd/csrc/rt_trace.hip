// rt_trace.hip — gfx950 path-trace kernel for the reference's per-pixel
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
// (compute_dynamic_ray.comp:185-210) node for node.
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

template <bool COUNT>
__global__ __launch_bounds__(256) void trace_kernel(TraceArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    // One wave = one 8x8 pixel tile (the reference's local_size 8x8x1,
    // compute_dynamic_ray.comp:157); a 256-thread block = 16x16 pixels.
    const int lx = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int ly = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    const bool active = lx < a.tw && ly < a.th;

    unsigned long long c_seg = 0, c_node = 0, c_tri = 0, c_mat = 0;

    if (active) {
        const int x = a.x0 + lx;
        const int y = a.y0 + ((ly / a.band_h) * a.band_stride + a.band_off) * a.band_h + ly % a.band_h;
        const float4* __restrict__ nodes = a.scene.nodes;
        const float4* __restrict__ tris  = a.scene.tris;
        const float4* __restrict__ mats  = a.scene.mats;
        const int end = a.scene.end;

        uint32_t seed = (uint32_t)(y * a.width + x);                                 // :164
        const float u = ((float)x + rnd(seed)) / (float)a.width;                     // :167
        const float v = ((float)(a.height - 1 - y) + rnd(seed)) / (float)a.height;   // :168

        const V3 cam_o = {a.cam.ox, a.cam.oy, a.cam.oz};
        const V3 cam_l = {a.cam.lx, a.cam.ly, a.cam.lz};
        const V3 cam_h = {a.cam.hx, a.cam.hy, a.cam.hz};
        const V3 cam_v = {a.cam.vx, a.cam.vy, a.cam.vz};
        V3 o = cam_o;
        V3 d = vnormalize(vsub(vadd(vadd(cam_l, vscale(cam_h, u)), vscale(cam_v, v)), cam_o));  // :173

        V3 fin = {0.0f, 0.0f, 0.0f};
        V3 att = {1.0f, 1.0f, 1.0f};

        for (int b = 0; b < a.max_bounces; ++b) {                                     // :179
            if (COUNT) ++c_seg;
            float closest = kTMax;
            int   hit = -1;
            V3    n = {0.0f, 0.0f, 0.0f};
            const V3 inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};                     // :89

            int i = 0;
            while (i < end) {
                const float4 A = nodes[2 * i];
                const float4 B = nodes[2 * i + 1];
                if (COUNT) ++c_node;
                // hit_aabb (:88-103)
                const float t0x = (A.x - o.x) * inv.x, t1x = (B.x - o.x) * inv.x;
                const float t0y = (A.y - o.y) * inv.y, t1y = (B.y - o.y) * inv.y;
                const float t0z = (A.z - o.z) * inv.z, t1z = (B.z - o.z) * inv.z;
                const float te = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
                const float tx = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
                const bool hb = tx > te && tx > kTMin && te < closest;
                const int leaf = __float_as_int(B.w);
                if (hb && leaf >= 0) {
                    if (COUNT) ++c_tri;
                    // hit_triangle (:105-129)
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
                                    n = {P0.w, P1.w, P2.w};
                                    if (vdot(d, n) > 0.0f) n = {-n.x, -n.y, -n.z};
                                }
                            }
                        }
                    }
                }
                i = hb ? i + 1 : __float_as_int(A.w);
            }

            if (hit >= 0) {                                                          // :212
                if (COUNT) ++c_mat;
                const V3 hp = vadd(o, vscale(d, closest));                             // ray_at :77-79
                const float4 M = mats[hit];
                bool scattered;
                V3 nd;
                if (M.w == 0.0f) {                                                   // Lambertian :137-143
                    const V3 ru = vnormalize(rnd_in_sphere(seed));
                    V3 sd = vadd(n, ru);
                    if (sqrtf(vdot(sd, sd)) < 0.0001f) sd = n;
                    nd = vnormalize(sd);
                    scattered = true;
                } else if (M.w == 1.0f || M.w == 2.0f) {                             // metal :145-151
                    const float fuzz = (M.w == 2.0f) ? 0.3f : 0.0f;
                    const V3 di = vnormalize(d);
                    const float k = 2.0f * vdot(n, di);
                    const V3 refl = vsub(di, vscale(n, k));                          // reflect()
                    const V3 p = rnd_in_sphere(seed);
                    nd = vnormalize(vadd(refl, vscale(p, fuzz)));
                    scattered = vdot(nd, n) > 0.0f;
                } else {
                    scattered = false;                                               // :153
                    nd = d;
                }
                if (scattered) {
                    att = vmul(att, V3{M.x, M.y, M.z});
                    o = hp;
                    d = nd;
                } else {
                    att = {0.0f, 0.0f, 0.0f};
                    break;
                }
            } else {
                // getSkyColor (:81-85)
                const V3 ud = vnormalize(d);
                const float t = 0.5f * (ud.y + 1.0f);
                const float omt = 1.0f - t;
                const V3 sky = {omt * 1.0f + t * 0.5f, omt * 1.0f + t * 0.7f, omt * 1.0f + t * 1.0f};
                fin = vmul(att, sky);
                break;
            }
            if (b == a.max_bounces - 1) fin = {0.0f, 0.0f, 0.0f};                   // :229-231
        }

        const V3 g = {sqrtf(fin.x), sqrtf(fin.y), sqrtf(fin.z)};                    // :235
        const size_t p = (size_t)ly * (size_t)a.tw + (size_t)lx;
        if (a.out_rgba) a.out_rgba[p] = make_uchar4(unorm8(g.x), unorm8(g.y), unorm8(g.z), 255);
        if (a.out_rad) {
            a.out_rad[3 * p + 0] = g.x;
            a.out_rad[3 * p + 1] = g.y;
            a.out_rad[3 * p + 2] = g.z;
        }
    }

    if (COUNT) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            c_seg  += __shfl_xor(c_seg, off);
            c_node += __shfl_xor(c_node, off);
            c_tri  += __shfl_xor(c_tri, off);
            c_mat  += __shfl_xor(c_mat, off);
        }
        if (lane == 0) {
            atomicAdd(&a.counters->segments, c_seg);
            atomicAdd(&a.counters->node_visits, c_node);
            atomicAdd(&a.counters->tri_tests, c_tri);
            atomicAdd(&a.counters->mat_reads, c_mat);
        }
    }
}

}  // namespace

hipError_t launch_trace(const TraceArgs& a, hipStream_t stream) {
    const dim3 block(256);
    const dim3 grid((a.tw + 15) / 16, (a.th + 15) / 16);
    if (a.counters)
        hipLaunchKernelGGL(trace_kernel<true>, grid, block, 0, stream, a);
    else
        hipLaunchKernelGGL(trace_kernel<false>, grid, block, 0, stream, a);
    return hipGetLastError();
}

}  // namespace rtamd
