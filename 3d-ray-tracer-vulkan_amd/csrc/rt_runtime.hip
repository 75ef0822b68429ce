// rt_runtime.hip — the C ABI of include/rtamd.h: context, scene upload and
// frame render.  Replaces the render-side role of VulkanEngine
// (VulkanEngine.java:318-431); the Vulkan plumbing (instance, descriptor sets,
// barriers, staging image) has no counterpart: device buffers + one HIP
// stream per device.
#include "rt_internal.h"
#include <rocprim/device/device_scan.hpp>

#include "accel_build.h"

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

namespace rtamd {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

#define RT_HIP_CHECK(expr)                                                        \
    do {                                                                          \
        hipError_t e_ = (expr);                                                   \
        if (e_ != hipSuccess) {                                                   \
            set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),      \
                      __FILE__, __LINE__);                                        \
            return RT_ERR_HIP;                                                    \
        }                                                                         \
    } while (0)

// ------------------------------------------------------------ scene build --

// The accel records' slot cap: 0 = the hardware's (accel_build.h).  Tests
// lower it through RTAMD_ACCEL_CAP_SLOTS to drive the capacity fallback.
static int64_t accel_cap_slots() {
    const char* v = std::getenv("RTAMD_ACCEL_CAP_SLOTS");
    return v ? std::atoll(v) : 0;
}

static inline float f32_at(const unsigned char* p, size_t off) {
    float f;
    std::memcpy(&f, p + off, 4);
    return f;
}
static inline int32_t i32_at(const unsigned char* p, size_t off) {
    int32_t v;
    std::memcpy(&v, p + off, 4);
    return v;
}

void free_host_scene(HostScene* s) {
    std::free(s->nodes);
    std::free(s->leafs);
    std::free(s->pairs);
    std::free(s->norms);
    std::free(s->mats);
    *s = HostScene{};
}

int build_host_scene(const void* vertices, size_t vertex_bytes,
                     const void* materials, size_t material_bytes,
                     const void* bvh_nodes, size_t bvh_bytes,
                     HostScene* out, const char** err) {
    static thread_local std::string msg;
    *out = HostScene{};
    const size_t n_nodes = bvh_bytes < RT_NODE_RECORD_BYTES ? 0 : bvh_bytes / RT_NODE_RECORD_BYTES;
    const size_t n_tris  = vertex_bytes < RT_VERTEX_RECORD_BYTES ? 0 : vertex_bytes / RT_VERTEX_RECORD_BYTES;
    const size_t n_mats  = material_bytes < RT_MATERIAL_RECORD_BYTES ? 0 : material_bytes / RT_MATERIAL_RECORD_BYTES;
    auto fail = [&](const std::string& m) {
        msg = m;
        *err = msg.c_str();
        free_host_scene(out);
        return RT_ERR_BAD_SCENE;
    };
    if (n_nodes && bvh_bytes % RT_NODE_RECORD_BYTES)
        return fail("bvh_bytes is not a multiple of 48");
    if (n_tris && vertex_bytes % RT_VERTEX_RECORD_BYTES)
        return fail("vertex_bytes is not a multiple of 48");
    if (n_mats && material_bytes % RT_MATERIAL_RECORD_BYTES)
        return fail("material_bytes is not a multiple of 16");
    if (n_nodes > (size_t)INT32_MAX / 2 || n_tris > (size_t)INT32_MAX / 3)
        return fail("scene too large for 32-bit node/triangle indices");
    if (n_nodes && (!bvh_nodes)) return fail("null bvh buffer");
    if (n_tris && (!vertices)) return fail("null vertex buffer");
    if (n_mats && (!materials)) return fail("null material buffer");

    out->n_nodes = (int)n_nodes;
    out->n_tris  = (int)n_tris;
    if (n_nodes == 0) {
        out->end = 0;   // empty scene: every ray misses (reference: undefined read of node 0)
        return RT_OK;
    }
    const unsigned char* nb = static_cast<const unsigned char*>(bvh_nodes);
    std::vector<int32_t> skip(n_nodes), depth(n_nodes, 0);
    out->nodes = static_cast<float4*>(std::malloc(sizeof(float4) * 2 * n_nodes));
    if (!out->nodes) return fail("out of host memory");

    // Pass 1 (reverse): leaf skip = i+1, internal skip = skip(right).  The
    // layout must be the reference flattener's preorder: left == i+1 and the
    // left subtree ends exactly where the right child starts.
    for (size_t k = n_nodes; k-- > 0;) {
        const unsigned char* r = nb + k * RT_NODE_RECORD_BYTES;
        const int32_t data = i32_at(r, 32), count = i32_at(r, 36);
        if (count < 0) {                                   // leaf (compute_dynamic_ray.comp:194-195)
            const int64_t tri = -((int64_t)data + 1);
            if (tri < 0 || (size_t)tri >= n_tris || (size_t)tri >= n_mats)
                return fail("leaf node " + std::to_string(k) + " references triangle " +
                            std::to_string(tri) + " outside the vertex/material buffers");
            skip[k] = (int32_t)(k + 1);
        } else {
            if ((size_t)data != k + 1 || count <= data || (size_t)count >= n_nodes)
                return fail("node " + std::to_string(k) +
                            " is not in the reference's preorder layout (left must be i+1, right > left)");
            if (skip[data] != count)
                return fail("node " + std::to_string(k) + ": left subtree does not end at the right child");
            skip[k] = skip[count];
        }
    }
    out->end = skip[0];
    std::vector<uint8_t> is_leaf(n_nodes + 1, 0);
    for (size_t k = 0; k < n_nodes; ++k) is_leaf[k] = i32_at(nb + k * RT_NODE_RECORD_BYTES, 36) < 0;
    out->root_leaf = is_leaf[0];
    out->leafs = static_cast<float4*>(std::calloc(3 * n_nodes, sizeof(float4)));
    out->pairs = static_cast<float4*>(std::calloc(4 * n_nodes, sizeof(float4)));
    if (!out->leafs || !out->pairs) return fail("out of host memory");
    const unsigned char* vb = static_cast<const unsigned char*>(vertices);
    int max_depth = 0;
    for (size_t k = 0; k < (size_t)out->end; ++k) {
        const unsigned char* r = nb + k * RT_NODE_RECORD_BYTES;
        const int32_t data = i32_at(r, 32), count = i32_at(r, 36);
        if (count >= 0) {
            depth[data] = depth[k] + 1;
            depth[count] = depth[k] + 1;
        }
        if (depth[k] > max_depth) max_depth = depth[k];
        float4 A, B;
        A.x = f32_at(r, 0);  A.y = f32_at(r, 4);  A.z = f32_at(r, 8);
        B.x = f32_at(r, 16); B.y = f32_at(r, 20); B.z = f32_at(r, 24);
        const uint32_t sk = (uint32_t)skip[k];
        const uint32_t aw = sk | ((sk < (uint32_t)out->end && is_leaf[sk]) ? 0x80000000u : 0u);
        const uint32_t bw = ((k + 1 < (size_t)out->end && is_leaf[k + 1]) ? 1u : 0u) | (is_leaf[k] ? 2u : 0u);
        std::memcpy(&A.w, &aw, 4);
        std::memcpy(&B.w, &bw, 4);
        out->nodes[2 * k] = A;
        out->nodes[2 * k + 1] = B;
        if (k == 0) {
            out->root_box[0] = A.x; out->root_box[1] = A.y; out->root_box[2] = A.z;
            out->root_box[3] = B.x; out->root_box[4] = B.y; out->root_box[5] = B.z;
        }
        if (count >= 0) {
            const unsigned char* l = nb + (size_t)data * RT_NODE_RECORD_BYTES;
            const unsigned char* rr = nb + (size_t)count * RT_NODE_RECORD_BYTES;
            const uint32_t rw = (uint32_t)count | (is_leaf[count] ? 0x80000000u : 0u);
            const uint32_t lw = is_leaf[data] ? 1u : 0u;
            const uint32_t sw = (uint32_t)skip[k];
            float rwf, lwf, swf;
            std::memcpy(&rwf, &rw, 4);
            std::memcpy(&lwf, &lw, 4);
            std::memcpy(&swf, &sw, 4);
            out->pairs[4 * k + 0] = make_float4(f32_at(l, 0), f32_at(l, 4), f32_at(l, 8), f32_at(rr, 0));
            out->pairs[4 * k + 1] = make_float4(f32_at(l, 16), f32_at(l, 20), f32_at(l, 24), f32_at(rr, 4));
            out->pairs[4 * k + 2] = make_float4(f32_at(rr, 16), f32_at(rr, 20), f32_at(rr, 24), f32_at(rr, 8));
            out->pairs[4 * k + 3] = make_float4(rwf, lwf, swf, 0.f);
        }
        if (count < 0) {
            // edge1 / edge2 exactly as hit_triangle computes them (compute_dynamic_ray.comp:106-107)
            const int32_t tri = -(data + 1);
            const unsigned char* v = vb + (size_t)tri * RT_VERTEX_RECORD_BYTES;
            const float v0x = f32_at(v, 0),  v0y = f32_at(v, 4),  v0z = f32_at(v, 8);
            const float v1x = f32_at(v, 16), v1y = f32_at(v, 20), v1z = f32_at(v, 24);
            const float v2x = f32_at(v, 32), v2y = f32_at(v, 36), v2z = f32_at(v, 40);
            float tw;
            std::memcpy(&tw, &tri, 4);
            out->leafs[3 * k + 0] = make_float4(v0x, v0y, v0z, tw);
            out->leafs[3 * k + 1] = make_float4(v1x - v0x, v1y - v0y, v1z - v0z, 0.f);
            out->leafs[3 * k + 2] = make_float4(v2x - v0x, v2y - v0y, v2z - v0z, 0.f);
        }
    }
    out->max_depth = max_depth;

    out->norms = static_cast<float4*>(std::malloc(sizeof(float4) * (n_tris ? n_tris : 1)));
    out->mats = static_cast<float4*>(std::malloc(sizeof(float4) * (n_tris ? n_tris : 1)));
    if (!out->norms || !out->mats) return fail("out of host memory");
    const unsigned char* mb = static_cast<const unsigned char*>(materials);
    for (size_t t = 0; t < n_tris; ++t) {
        const unsigned char* r = vb + t * RT_VERTEX_RECORD_BYTES;
        const float v0x = f32_at(r, 0),  v0y = f32_at(r, 4),  v0z = f32_at(r, 8);
        const float v1x = f32_at(r, 16), v1y = f32_at(r, 20), v1z = f32_at(r, 24);
        const float v2x = f32_at(r, 32), v2y = f32_at(r, 36), v2z = f32_at(r, 40);
        // normalize(cross(edge1, edge2)) exactly as hit_triangle computes it (:124)
        const float e1x = v1x - v0x, e1y = v1y - v0y, e1z = v1z - v0z;
        const float e2x = v2x - v0x, e2y = v2y - v0y, e2z = v2z - v0z;
        const float cx = e1y * e2z - e1z * e2y;
        const float cy = e1z * e2x - e1x * e2z;
        const float cz = e1x * e2y - e1y * e2x;
        const float l = std::sqrt((cx * cx + cy * cy) + cz * cz);
        out->norms[t] = make_float4(cx / l, cy / l, cz / l, 0.f);
        if (t < n_mats) {
            const unsigned char* m = mb + t * RT_MATERIAL_RECORD_BYTES;
            out->mats[t] = make_float4(f32_at(m, 0), f32_at(m, 4), f32_at(m, 8), f32_at(m, 12));
        } else {
            out->mats[t] = make_float4(0.f, 0.f, 0.f, -1.f);   // never referenced (validated above)
        }
    }
    return RT_OK;
}

}  // namespace rtamd

// ------------------------------------------------------------------ context --

using namespace rtamd;

static constexpr int kMaxSlots = 8;   // rt_render_async frame slots per device
// Walk records with no leaf straddling a 128-B line (option leaf_align; 2 =
// auto: aligned when the packed records exceed kWin32Bytes, like the window
// size): config 5 8.24 vs 8.39-8.46 ms and 21.3 vs 22.4 GB fetched per frame
// (profiles/r04/r4g), for 11% more slots.  A scene whose records stay in L2
// gains nothing from it, and its kernels then skip the pad-bit arithmetic
// (kFeatPad off: config 3 0.303-0.304 vs 0.306-0.307 ms, profiles/r04/r4m).
#ifndef RT_LEAF_ALIGN
#define RT_LEAF_ALIGN 2
#endif
// Option accel's default: the binned-SAH tree in 8 octant
// layouts.  Config 3 0.1279-0.1288 ms per frame against 0.2962-0.2964 for the
// reference's tree and order, config 5 1.24-1.25 against 7.84 ms, config 6
// 0.140 against 0.342 (profiles/r05/r5a, r5b); 1 layout: 0.1365, 1.40, 0.148.
#ifndef RT_ACCEL
#define RT_ACCEL 8
#endif
// Option accel_half's default: the accel records' internal boxes in half
// precision (accel_build.h format 1).
#ifndef RT_ACCEL_HALF
#define RT_ACCEL_HALF 0
#endif
// Option accel_wide's default: the 4-wide tree (accel_build.h format 2).
#ifndef RT_ACCEL_WIDE
#define RT_ACCEL_WIDE 0
#endif
// Option split_bounce's default.
#ifndef RT_SPLIT_BOUNCE
#define RT_SPLIT_BOUNCE 0
#endif

struct PerDevice {
    int          device = 0;
    hipStream_t  stream = nullptr;
    hipEvent_t   ev0 = nullptr, ev1 = nullptr;
    DevScene     scene;
    Counters*    d_counters = nullptr;
    uchar4*      d_rgba = nullptr;
    float*       d_rad = nullptr;
    size_t       out_cap = 0;      // pixels
    unsigned long long* d_diag = nullptr;   // diagnostics (option "diag")
    size_t       diag_cap = 0, diag_used = 0;
    int          n_cu = 0;
    // rt_render_async: frame slots (option async_slots), each with its own
    // trace stream, one copy stream (two for a one-device frame, option
    // copy_streams), per-slot events and the last ticket of a slot
    hipStream_t  copy_stream = nullptr, copy_stream2 = nullptr;
    uchar4*      d_ring[kMaxSlots] = {};
    size_t       ring_cap = 0;     // pixels per slot
    hipStream_t  slot_stream[kMaxSlots] = {};
    hipEvent_t   traced[kMaxSlots] = {}, copied[kMaxSlots] = {}, copied2[kMaxSlots] = {};
    uint64_t     slot_ticket[kMaxSlots] = {};
    bool         slot_split[kMaxSlots] = {};   // the slot's newest frame split its readback (copy_stream2)
    uint64_t     last_split_t = 0;             // newest split frame's ticket, its copied2 slot
    int          last_split_slot = -1;
    float*       d_accum = nullptr;  // extension kExtAccumulate: running sums
    float4*      d_spheres = nullptr; // extension kExtSpheres: 2 float4 per sphere
    int          n_spheres = 0;
    size_t       accum_n = 0;        // floats
    // option heavy_first: per-wave costs of a learning launch, and the tile
    // orders (most expensive first) learned so far, one per launch key (a
    // band partition rotates through several keys), oldest dropped first
    unsigned long long* d_learn = nullptr;   // per-wave diag records of the learning launch
    size_t       learn_cap = 0;
    unsigned*    d_learn_lane = nullptr;    // per-pixel walk lengths of the learning launch (64 per wave)
    size_t       learn_lane_cap = 0;
    // a learned order: tiles most expensive first, the heavy-tile count, and
    // the heavy pixels (tile * 64 + lane, most expensive first) with every
    // tile's mask of them (option heavy_pixels)
    struct Order { std::vector<uint8_t> key; int* d_order; size_t n; int heavy;
                   int* d_hpix; int n_hpix; unsigned long long* d_mask;
                   bool pending = false;      // learned on the device, heavy-pixel count not read yet
                   void* d_base = nullptr;    // one allocation holding d_order, d_mask, d_hpix, d_nhpix
                   int* d_nhpix = nullptr; };
    // device-side learning (rt_learn.hip): one at a time per device; its
    // scratch, the pinned heavy-pixel count it reports and the event after it
    void*        d_learn_scratch = nullptr;
    size_t       learn_scratch_cap = 0;
    int*         h_nhpix = nullptr;           // pinned
    hipEvent_t   learn_ev = nullptr;
    bool         learn_busy = false;          // a device learning is in flight (its order pending)
    bool         learn_oom = false;           // device learning's scratch did not fit: learn on the host
    bool         learning_device = false;     // the learning launch being planned learns on the device
    int          learning_rec_off = 0;        // its heavy-pixel waves ahead of the tile records
    // option heavy_tiles: auxiliary streams (round robin) for the concurrent heavy-tile launch
    hipStream_t  aux[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t   aux_fork[4] = {nullptr, nullptr, nullptr, nullptr}, aux_join[4] = {nullptr, nullptr, nullptr, nullptr};
    unsigned     aux_next = 0;
    std::vector<Order> orders;
    std::vector<uint8_t> learning_key;
    // option reuse_order: the camera of the last heavy_first launch of each
    // frame geometry + scene (key without its camera bytes), newest last, so
    // several geometries interleaved on one device (band offsets, rotating
    // pieces, callers' streams) each see their own camera stop
    struct LastCam { std::vector<uint8_t> geo; std::vector<uint8_t> cam; };
    std::vector<LastCam> last_cam;
    size_t       learning_n = 0;
    int          learning_tx = 0, learning_ty = 0, learning_frames = 0;   // its tiles (option xcd_order)
    int          last_heavy = 0;    // heavy tiles of the last launch (option "heavy_tiles_used", read only)
    int          last_heavy_px = 0; // heavy pixels of the last launch (option "heavy_pixels_used", read only)
    // option graph: plain launches captured once per launch key into a HIP
    // graph and replayed (the heavy-tile fork / join becomes graph edges)
    struct Graph { std::vector<uint64_t> key; hipGraphExec_t exec; int kernels; };
    uint64_t     plain_kernels = 0;  // production-build kernels enqueued (option "plain_kernels", read only)
    struct BandList { std::vector<int> bands; int* d; };
    std::vector<BandList> band_lists;   // rt_render_batch_device's band lists on this device
    std::vector<Graph> graphs;
    unsigned     graph_next = 0;
    // option split_bounce: one set of ray slots per launch stream (rt_internal.h
    // TraceArgs::q_slots), grown to the largest launch seen on that stream
    struct Slots { hipStream_t s; char* base; int waves; size_t temp_bytes; };
    std::vector<Slots> slots;
};

static constexpr size_t kMaxOrders = 16;
static constexpr int    kResidentPerCu = 24;    // resident trace waves per CU (diag timelines)
static constexpr int    kMaxHeavy = 256;
// coop_window 0: scenes whose walk records exceed the 8 XCDs' L2s together
// (8 x 4 MB) take 32-slot windows: config 5 (100 MB) fetched 22.4 instead of
// 28.5 GB per frame at the same frame time; config 3 (6.3 MB, L2-resident)
// is 1.2% faster with 64 (profiles/r04/r4f).
static constexpr size_t kWin32Bytes = 32ull << 20;
// option split_bounce: the largest ray-slot allocation per launch stream
static constexpr size_t kSplitSlotBytes = 256ull << 20;
// The walk's buffer loads address the records with 32-bit byte offsets
// (rt_trace.hip, RT_CHAIN 2): at most 2^27 - 4 slots of 32 B (~45M triangles).
static constexpr unsigned kMaxWalkSlots = (1u << 27) - 4;
static constexpr size_t kDiagWords = 8;   // per-wave diag record (rt_trace.hip, rtamd.h rt_diag_copy)

static void free_order(PerDevice::Order& o) {
    if (o.d_base) {                              // device-learned: one allocation
        (void)hipFree(o.d_base);
        return;
    }
    (void)hipFree(o.d_order);
    if (o.d_hpix) (void)hipFree(o.d_hpix);
    if (o.d_mask) (void)hipFree(o.d_mask);
}

// A device learning in flight: once its event has fired, its order's
// heavy-pixel count (copied to pinned memory by the same stream) is read and
// the order becomes usable.  Never blocks.
static void poll_learning(PerDevice& p) {
    if (!p.learn_busy || hipEventQuery(p.learn_ev) != hipSuccess) return;
    for (auto& o : p.orders)
        if (o.pending) {
            o.n_hpix = std::max(0, *p.h_nhpix);
            o.pending = false;
        }
    p.learn_busy = false;
}

static void free_orders(PerDevice& p) {
    for (auto& o : p.orders) free_order(o);
    p.orders.clear();
}

static void free_graphs(PerDevice& p) {
    for (auto& g : p.graphs) (void)hipGraphExecDestroy(g.exec);
    p.graphs.clear();
}
static constexpr size_t kMaxGraphs = 64;   // an 8-rank frame batch with two buffers uses 16 keys

static constexpr size_t kMaxLastCams = 64;

struct rt_ctx {
    std::vector<PerDevice> dev;
    int  wave_tile = -1;           // 8x8 / 16x4 / 32x2 / 64x1 pixels per wave (0-3); -1 (default) = 16x4
                                   //   when the walk records exceed kWin32Bytes, else 8x8
    int  diag = 0;                 // record per-wave timestamps
    int  coop_lanes = -1;          // cooperative tail once <= this many lanes walk (0 = off); -1 (default) =
                                   //   1 on the reference-order walk, 0 on the accel walk (its walks are
                                   //   short: config 3 0.1253-0.1254 vs 0.1279-0.1288 ms, profiles/r05/r5b)
    int  ext = 0;                  // non-reference extensions (kExt* bits), off by default
    int  walk = 2;                 // 0 = node per step, 2 = node per step, software-pipelined over the
                                   //   compact records (fastest measured)
    int  coop_walk = 0;            // cooperative walks: 0 = 64-node windows, 1 = preorder frontier
    int  coop_window = 0;          // coop_walk's window: 64 or 32 slots; 0 = 32 when the walk records
                                   //   exceed kWin32Bytes (they cannot stay in the L2s), else 64
    int  block_waves = 1;          // waves per workgroup (1: a finished wave frees its slot at once; or 4)
    int  heavy_first = 1;          // dispatch tiles in the cost order of a learning launch
    int  heavy_factor = 130;       // automatic heavy tiles: walk length above this percentage of the bulk estimate
    int  heavy_pixels = 1;         // heavy_stream 2 with automatic heavy tiles: split heavy PIXELS (1) or
                                   //   whole tiles (0) into one-pixel waves
    int  heavy_pixel_factor = 50;  // heavy pixels: walk length above this percentage of the bulk estimate
    int  reuse_order = 1;          // heavy_first: a moving camera reuses the order learned at another camera
    int  heavy_cap = 75;           // automatic heavy tiles: at most this percentage of one generation of
                                   //   one-pixel waves (CUs x 24 / 64 tiles)
    int  async_slots = 4;          // rt_render_async: frames in flight per device, each on its own stream
    int  copy_streams = 1;         // rt_render_async, one device: the readback split over this many copy streams (2 measured slower)
    int  in_async = 0;             // set while rt_render_async plans a launch: its frames in flight
    int  concurrent_launches = 1;  // launches of similar work the caller keeps in flight on a device at once
                                   //   (the heavy-tile bulk estimate counts this launch's work that many times)
    int  learn_cost = 1;           // heavy_first cost: 0 = lockstep steps + 2 x coop windows, 1 = wave duration
    int  learn_alone = 0;          // heavy_first: a learning launch first waits for the device to drain
    int  accel_octants = 7;        // option accel (8 layouts): the octant bits a ray's layout keeps
    int  xcd_order = 0;            // device-learned orders: XCD c takes one class of row bands (rt_learn.hip;
                                   //   the band height in wave-tile rows, 0 = off)
    int  learn_device = 1;         // heavy_first: learn the order on the device (rt_learn.hip; 0 = on the host)
    int  leaf_align = RT_LEAF_ALIGN;   // walk records: no leaf straddles a 128-B line (a pad slot before it)
    int  accel_half = RT_ACCEL_HALF;   // at the next upload: accel records in format 1 (accel_build.h)
    int  accel_wide = RT_ACCEL_WIDE;   // at the next upload: the 4-wide tree, format 2 (overrides accel_half)
    int  split_bounce = RT_SPLIT_BOUNCE;   // accel walk: paths alive at this bounce finish in a second kernel
                                   //   (0 = one kernel)
    int  accel = RT_ACCEL;         // at the next upload: 0 = the reference's tree and order; 1 / 8 = the
                                   //   SAH tree in 1 / 8 (octant) layouts (accel_build.h)
    int  order_split = 0;          // heavy_first: only tiles costing >= this percent of the costliest go first
                                   //   (in cost order); the rest keep their raster order (0 = all by cost)
    int  order_frames = 0;         // heavy_first, several frames per launch: the non-leading tiles row by row
                                   //   across the frames (0 = frame by frame)
    int  graph = 1;                // kernel 0 plain launches: replay a captured HIP graph per launch key
    int  heavy_stream = 2;         // heavy_tiles: 1 = their launch runs on an auxiliary stream, concurrent
                                   //   with the other tiles; 2 = their workgroups come first in the
                                   //   other tiles' launch (one launch per frame)
                                   //   with the other tiles; 0 = before them on the same stream
    int  heavy_tiles = -1;         // heavy_first: the this-many most expensive tiles are traced one pixel
                                   //   per wave, walked cooperatively, in a separate launch
                                   //   (-1 = automatic: the tiles that outlast the bulk, learn_order)
    uint64_t scene_gen = 0;        // bumped by every scene upload (invalidates learned tile orders)
    int  hw_queues = 4;            // GPU_MAX_HW_QUEUES seen at rt_create (HIP's default 4); frames in
                                   //   flight on more streams than queues - 2 share queues and serialise
    bool has_scene = false;
    int  n_nodes = 0, n_tris = 0, max_depth = 0;
    uint64_t issued = 0;           // rt_render_async tickets handed out
};

static void free_scene(PerDevice& p) {
    if (p.scene.nodes) (void)hipFree(p.scene.nodes);
    if (p.scene.leafs) (void)hipFree(p.scene.leafs);
    if (p.scene.walk) (void)hipFree(p.scene.walk);
    if (p.scene.walk_ref) (void)hipFree(p.scene.walk_ref);
    if (p.scene.slot_node) (void)hipFree(p.scene.slot_node);
    if (p.scene.node_slot) (void)hipFree(p.scene.node_slot);
    if (p.scene.pairs) (void)hipFree(p.scene.pairs);
    if (p.scene.norms) (void)hipFree(p.scene.norms);   // mats lives in the same allocation
    p.scene = DevScene{};
}

// Launches of similar work on a device at once, for the heavy-pixel bar: the
// caller's statement (option concurrent_launches), or rt_render_async's own
// frames in flight.
static int concurrency(const rt_ctx* ctx) { return std::max(ctx->concurrent_launches, ctx->in_async); }

// Heavy-first dispatch (option heavy_first, kernel 0 with one-wave
// workgroups): the first launch of a given frame geometry + camera + scene
// records every wave's duration; the host sorts the tiles by it, most
// expensive first, and later launches with the same key dispatch in that
// order, so the waves that set the frame time start first.  Results do not
// change (a tile's pixels and seeds are the same whichever workgroup traces
// it); the learning launch ends with a stream synchronisation.
static int plan_order(const rt_ctx* ctx, PerDevice& p, TraceArgs& a, const rt_camera_ubo* cams,
                      const std::vector<int>* bands) {
    a.tile_order = nullptr;
    a.tiles_x = 0;
    a.split_n = 0;
    a.heavy_tiles = 0;
    a.aux_stream = nullptr;
    a.heavy_fused = 0;
    a.heavy_px = nullptr;
    a.n_heavy_px = 0;
    a.tile_mask = nullptr;
    a.diag_lane = nullptr;
    a.ev_fork = a.ev_join = nullptr;
    p.last_heavy = 0;
    p.last_heavy_px = 0;
    if (!ctx->heavy_first || a.block_waves != 1) return RT_OK;
    const int tw_w = 8 << a.wave_tile, th_w = 8 >> a.wave_tile, bw = a.block_waves;
    // every frame of a batch has the same tiles; the order covers all of them
    const size_t n = (size_t)((a.tw + bw * tw_w - 1) / (bw * tw_w)) * bw * (size_t)((a.th + th_w - 1) / th_w) *
                     (size_t)a.n_frames;
    // key = geometry (+ the band list) | the cameras | the scene
    // (the heavy-split options are part of the key: an order learned on the
    // device has no heavy tiles, one learned on the host does)
    std::vector<int> geo = {a.width, a.height, a.max_bounces, a.x0, a.y0, a.tw, a.th, a.band_h, a.band_stride,
                            a.band_off, a.wave_tile, a.ext, a.coop_lanes, a.walk, ctx->learn_cost, ctx->order_split,
                            ctx->heavy_factor, concurrency(ctx), ctx->heavy_cap, ctx->heavy_pixel_factor,
                            a.n_frames, bands ? (int)bands->size() : -1, a.list_stride, ctx->order_frames,
                            ctx->heavy_stream, ctx->heavy_pixels, ctx->heavy_tiles, ctx->learn_device,
                            ctx->xcd_order, ctx->accel_octants};
    if (bands) geo.insert(geo.end(), bands->begin(), bands->end());
    const size_t g = geo.size() * sizeof(int), c = (size_t)a.n_frames * sizeof(rt_camera_ubo);
    std::vector<uint8_t> key(g + c + sizeof(uint64_t));
    std::memcpy(key.data(), geo.data(), g);
    std::memcpy(key.data() + g, cams, c);
    std::memcpy(key.data() + g + c, &ctx->scene_gen, sizeof(uint64_t));
    // Use a learned order: the exact key's; or, when only the camera differs
    // from a learned key and the camera has just moved (option reuse_order),
    // the newest order of the same frame geometry and scene.  The order and the
    // heavy pixels only decide which wave traces a pixel and when, never what
    // it computes, so an order learned at another camera is exact, only less
    // well balanced; a camera in motion pays no learning frame, and the first
    // repeat of a camera (the camera has stopped) learns its own order.
    // Heavy pixels / tiles are split out only where the launcher can do it:
    // the cooperative tail on and no extensions (the one-pixel waves are a
    // branch of the cooperative-tail kernel), and for the fused launch
    // (heavy_stream 2) the default walk 2, which that launch runs.  Otherwise
    // a launch uses the learned order alone (and reports no heavy work).
    const bool splittable = a.coop_lanes > 0 && a.ext == 0 && (ctx->heavy_stream != 2 || a.walk == 2) &&
                            a.scene.n_layouts == 0;   // accel: no frontier walk for heavy work
    auto use = [&](const PerDevice::Order& o) -> int {
        a.tile_order = o.d_order;
        if (!splittable) return RT_OK;
        if (ctx->heavy_stream == 2 && ctx->heavy_pixels && ctx->heavy_tiles < 0 && n > 1) {
            // heavy pixels, fused: their one-pixel workgroups come first
            // in the launch, and their tiles skip them
            a.heavy_fused = 1;
            a.heavy_px = o.d_hpix;
            a.n_heavy_px = o.n_hpix;
            a.tile_mask = o.d_mask;
            p.last_heavy_px = o.n_hpix;
            if (a.diag) p.diag_used = (n + (size_t)o.n_hpix) * 8;
            return RT_OK;
        }
        const int heavy = ctx->heavy_tiles >= 0 ? ctx->heavy_tiles : o.heavy;
        if (heavy > 0 && n > 1) {
            const unsigned k = p.aux_next++ % 4;
            if (!p.aux[k]) {
                // normal priority: a high-priority stream measured slower (0.715 vs 0.59 ms)
                RT_HIP_CHECK(hipStreamCreateWithFlags(&p.aux[k], hipStreamNonBlocking));
                RT_HIP_CHECK(hipEventCreateWithFlags(&p.aux_fork[k], hipEventDisableTiming));
                RT_HIP_CHECK(hipEventCreateWithFlags(&p.aux_join[k], hipEventDisableTiming));
            }
            a.heavy_tiles = heavy;
            p.last_heavy = (int)std::min<size_t>((size_t)heavy, n - 1);
            a.aux_stream = ctx->heavy_stream == 1 ? p.aux[k] : nullptr;
            a.heavy_fused = ctx->heavy_stream == 2 ? 1 : 0;
            a.ev_fork = p.aux_fork[k];
            a.ev_join = p.aux_join[k];
            if (a.diag)   // one record per workgroup of both launches
                p.diag_used = (n + 63 * (size_t)std::min(a.heavy_tiles, (int)n - 1)) * 8;
        }
        return RT_OK;
    };
    // Has the camera stopped?  Compared with the last launch of the same
    // frame geometry and scene, not with the device's last launch: several
    // geometries interleave on one device (band offsets, callers' streams).
    bool repeat = false;
    {
        std::vector<uint8_t> geo_scene(key.begin(), key.begin() + g);
        geo_scene.insert(geo_scene.end(), key.begin() + g + c, key.end());
        std::vector<uint8_t> camk(key.begin() + g, key.begin() + g + c);
        auto it = std::find_if(p.last_cam.begin(), p.last_cam.end(),
                               [&](const PerDevice::LastCam& l) { return l.geo == geo_scene; });
        if (it != p.last_cam.end()) {
            repeat = it->cam == camk;
            it->cam = std::move(camk);
            std::rotate(it, it + 1, p.last_cam.end());      // newest last
        } else {
            if (p.last_cam.size() >= kMaxLastCams) p.last_cam.erase(p.last_cam.begin());
            p.last_cam.push_back(PerDevice::LastCam{std::move(geo_scene), std::move(camk)});
        }
    }
    poll_learning(p);
    static const bool dbg = std::getenv("RTAMD_DEBUG_PLAN") != nullptr;
    const PerDevice::Order* exact = nullptr;
    for (const auto& o : p.orders)
        if (o.n == n && o.key == key) { exact = &o; break; }
    if (dbg) {
        size_t n_reuse = 0;
        for (const auto& o : p.orders)
            if (!o.pending && o.n == n && o.key.size() == key.size() && std::memcmp(o.key.data(), key.data(), g) == 0)
                ++n_reuse;
        std::fprintf(stderr, "plan_order: n %zu frames %d lists %d exact %d pending %d same-geo %zu repeat %d busy %d "
                     "orders %zu diag %d counters %d\n", n, a.n_frames, bands ? (int)bands->size() : -1,
                     exact != nullptr, exact ? (int)exact->pending : -1, n_reuse, (int)repeat, (int)p.learn_busy,
                     p.orders.size(), a.diag != nullptr, a.counters != nullptr);
    }
    if (exact && !exact->pending) {
        if (dbg) std::fprintf(stderr, "  -> exact order %p\n", (void*)exact->d_order);
        return use(*exact);
    }
    const PerDevice::Order* reuse = nullptr;
    if (ctx->reuse_order)
        for (auto it = p.orders.rbegin(); it != p.orders.rend(); ++it)
            if (!it->pending && it->n == n && it->key.size() == key.size() &&
                std::memcmp(it->key.data(), key.data(), g) == 0 &&
                std::memcmp(it->key.data() + g + c, key.data() + g + c, sizeof(uint64_t)) == 0) {
                reuse = &*it;
                break;
            }
    // A moving camera reuses the newest order of the frame geometry; so does
    // any launch while this key's own order is still being learned.
    if (reuse && (!repeat || exact)) {
        if (dbg) std::fprintf(stderr, "  -> reuse order %p\n", (void*)reuse->d_order);
        return use(*reuse);
    }
    if (exact) return RT_OK;                  // learning in flight, nothing to reuse: raster order
    // Learn on a plain launch: a diagnostic launch keeps its own records, and a
    // counting launch (stats) runs the counting build, not the diagnostic one.
    if (a.diag || a.counters) return RT_OK;
    // Device learning (rt_learn.hip), for the default heavy-pixel schedule: the
    // learning launch runs in the reused order if there is one (its heavy
    // pixels one per wave, as production launches), and the order is computed
    // on its stream afterwards with no synchronisation; one learning at a
    // time per device.  Other schedules learn on the host (learn_order).
    const bool device = ctx->learn_device && ctx->heavy_stream == 2 && ctx->heavy_pixels && ctx->heavy_tiles < 0 &&
                        !ctx->order_frames && !p.learn_oom;
    if (p.learn_busy) return reuse ? use(*reuse) : RT_OK;   // the device learning in flight finishes first
    // a fused launch's heavy-pixel waves record first: at most one per resident
    // wave slot (the largest cap any concurrency gives)
    const size_t recs = n + (device ? (size_t)p.n_cu * kResidentPerCu : 0);
    if (recs * kDiagWords > p.learn_cap) {
        if (p.d_learn) (void)hipFree(p.d_learn);
        p.d_learn = nullptr;
        p.learn_cap = 0;
        RT_HIP_CHECK(hipMalloc(&p.d_learn, recs * kDiagWords * sizeof(unsigned long long)));
        p.learn_cap = recs * kDiagWords;
    }
    if (n * 64 > p.learn_lane_cap) {
        if (p.d_learn_lane) (void)hipFree(p.d_learn_lane);
        p.d_learn_lane = nullptr;
        p.learn_lane_cap = 0;
        RT_HIP_CHECK(hipMalloc(&p.d_learn_lane, n * 64 * sizeof(unsigned)));
        p.learn_lane_cap = n * 64;
    }
    p.learning_key = key;
    p.learning_n = n;
    p.learning_tx = (a.tw + tw_w - 1) / tw_w;
    p.learning_ty = (a.th + th_w - 1) / th_w;
    p.learning_frames = a.n_frames;
    p.learning_device = device;
    p.learning_rec_off = 0;
    // Option learn_alone: the learning launch waits for the device to drain,
    // so its wave durations (the order's cost) are not those of waves that
    // shared the GPU with other launches in flight at that moment.
    if (ctx->learn_alone) RT_HIP_CHECK(hipDeviceSynchronize());
    if (device && reuse) {
        if (int rc = use(*reuse)) return rc;
        if (a.heavy_fused) p.learning_rec_off = a.n_heavy_px;
    }
    a.diag = p.d_learn;                // the diagnostic build counts each wave's lockstep steps
    a.diag_lane = p.d_learn_lane;      // and each pixel's own walk length
    if (dbg) std::fprintf(stderr, "  -> learn (device %d, in order %p)\n", (int)device, (void*)a.tile_order);
    return RT_OK;
}

// The device path of learn_order: a pending order whose buffers the learning
// kernels fill on stream s; the heavy-pixel count follows into pinned memory
// and an event marks it ready (poll_learning).
static int learn_order_device(const rt_ctx* ctx, PerDevice& p, hipStream_t s) {
    const size_t n = p.learning_n;
    const int conc = std::max(1, concurrency(ctx));
    const int cap = std::max(1, p.n_cu * kResidentPerCu * ctx->heavy_cap / 100 / conc);
    const size_t need = learn_scratch_bytes((int)n);
    // Out of device memory for the learning's scratch (it sorts a 64-bit key
    // per pixel): no order from this launch, and later launches learn on the
    // host (advisor, round 5: a plain render must not fail on it).
    const auto oom = [&p]() {
        (void)hipGetLastError();
        p.learn_oom = true;
        return RT_OK;
    };
    if (need > p.learn_scratch_cap) {
        if (p.d_learn_scratch) (void)hipFree(p.d_learn_scratch);
        p.d_learn_scratch = nullptr;
        p.learn_scratch_cap = 0;
        if (hipMalloc(&p.d_learn_scratch, need) != hipSuccess) return oom();
        p.learn_scratch_cap = need;
    }
    if (!p.h_nhpix) RT_HIP_CHECK(hipHostMalloc(&p.h_nhpix, sizeof(int), hipHostMallocPortable));
    if (!p.learn_ev) RT_HIP_CHECK(hipEventCreateWithFlags(&p.learn_ev, hipEventDisableTiming));
    if (p.orders.size() >= kMaxOrders) {
        RT_HIP_CHECK(hipDeviceSynchronize());  // the oldest order may still steer a launch in flight
        free_order(p.orders.front());
        p.orders.erase(p.orders.begin());
    }
    auto up = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t b_order = up(n * sizeof(int)), b_mask = up(n * sizeof(unsigned long long));
    const size_t b_hpix = up((size_t)cap * sizeof(int));
    PerDevice::Order o{p.learning_key, nullptr, n, 0, nullptr, 0, nullptr};
    if (hipMalloc(&o.d_base, b_order + b_mask + b_hpix + sizeof(int)) != hipSuccess) return oom();
    char* base = static_cast<char*>(o.d_base);
    o.d_order = reinterpret_cast<int*>(base);
    o.d_mask = reinterpret_cast<unsigned long long*>(base + b_order);
    o.d_hpix = reinterpret_cast<int*>(base + b_order + b_mask);
    o.d_nhpix = reinterpret_cast<int*>(base + b_order + b_mask + b_hpix);
    o.pending = true;
    LearnParams lp;
    lp.n = (int)n;
    lp.rec_off = p.learning_rec_off;
    lp.learn_cost = ctx->learn_cost;
    lp.order_split = ctx->order_split;
    // the host path's bar: heavy_pixel_factor% x (total steps x concurrent / resident waves)
    lp.bar_scale = ctx->heavy_pixel_factor / 100.0 * (double)conc / (double)std::max(1, p.n_cu * kResidentPerCu);
    lp.cap = cap;
    lp.xcd = ctx->xcd_order;
    lp.tiles_x = p.learning_tx;
    lp.tiles_y = p.learning_ty;
    lp.frames = p.learning_frames;
    hipError_t e = learn_on_device(lp, p.d_learn, p.d_learn_lane, p.d_learn_scratch, o.d_order, o.d_mask, o.d_hpix,
                                   o.d_nhpix, s);
    if (e == hipSuccess) e = hipMemcpyAsync(p.h_nhpix, o.d_nhpix, sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipEventRecord(p.learn_ev, s);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(s);
        free_order(o);
        RT_HIP_CHECK(e);
    }
    p.orders.push_back(std::move(o));
    p.learn_busy = true;
    return RT_OK;
}

// A tile's cost is its wave's lockstep walk iterations plus twice its
// cooperative windows (diag record words 4 and 5): the length of the wave's
// dependent chain, free of when the wave happened to run.
static int learn_order(const rt_ctx* ctx, PerDevice& p, const TraceArgs& a, hipStream_t s) {
    const int learn_cost = ctx->learn_cost, concurrent = concurrency(ctx);
    const double heavy_factor = ctx->heavy_factor / 100.0;
    if (!a.diag || a.diag != p.d_learn) return RT_OK;
    if (p.learning_device) return learn_order_device(ctx, p, s);
    const size_t n = p.learning_n;
    RT_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<unsigned long long> rec(n * kDiagWords);
    RT_HIP_CHECK(hipMemcpy(rec.data(), p.d_learn, rec.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    // Two costs per tile: its wave's duration (orders the tiles: it also sees
    // when and beside what the wave ran) and its lockstep steps + 2 x
    // cooperative windows (a deterministic walk length: counts the heavy tiles).
    std::vector<unsigned long long> cost(n), steps(n);
    for (size_t k = 0; k < n; ++k) {
        const unsigned long long* r = &rec[k * kDiagWords];
        steps[k] = r[4] + 2 * r[5];
        cost[k] = learn_cost == 0 ? steps[k] : r[1] - r[0];
    }
    std::vector<int> order(n);
    for (size_t k = 0; k < n; ++k) order[k] = (int)k;
    // Option order_split: the tiles that cost at least that percentage of the
    // costliest tile go first, most expensive first (they would otherwise end
    // the launch); the rest keep their raster order, so the waves running at
    // once trace neighbouring tiles of one frame (one BVH neighbourhood in the
    // caches) rather than tiles of like cost scattered over the launch's frames.
    unsigned long long cmax = 0;
    for (size_t k = 0; k < n; ++k) cmax = std::max(cmax, cost[k]);
    const double split_at = (double)ctx->order_split / 100.0 * (double)cmax;
    auto first = [&](int x) { return ctx->order_split == 0 || (double)cost[x] >= split_at; };
    auto mid = std::stable_partition(order.begin(), order.end(), first);
    std::stable_sort(order.begin(), mid, [&](int x, int y) { return cost[x] > cost[y]; });
    // Option order_frames (a launch of several frames): the rest go row by
    // row across the launch's frames (tile row y of frame 0, of frame 1, ...,
    // then row y + 1), so the waves running at once trace the same part of
    // the image in every frame of the batch instead of the rows of one or two
    // frames spread over a rank's band share.
    if (ctx->order_frames && a.n_frames > 1) {
        const int tw_w = 8 << a.wave_tile, th_w = 8 >> a.wave_tile;
        const long tx = (a.tw + tw_w - 1) / tw_w, ty = (a.th + th_w - 1) / th_w;
        auto key = [&](int k) {
            const long by = k / tx, f = by / ty, row = by % ty;
            return (row * a.n_frames + f) * tx + k % tx;
        };
        std::stable_sort(mid, order.end(), [&](int x, int y) { return key(x) < key(y); });
    }
    // Automatic heavy tiles: the tiles whose walk length exceeds heavy_factor
    // times the bulk estimate, the total walk length spread over the device's
    // resident waves (kResidentPerCu per CU, measured).  A 1080p frame of
    // config 3 gets a few dozen; a frame whose time is its throughput
    // (config 5) gets none.  The caller states how many launches of similar
    // work it keeps in flight on the device at once (option
    // concurrent_launches: bench.py's frame batches trace every band offset of
    // a frame concurrently, a render loop with frames in flight two or three);
    // the bulk counts this launch's work that many times.
    double total = 0.0;
    for (size_t k = 0; k < n; ++k) total += (double)steps[k];
    total *= (double)std::max(1, concurrent);
    const double bulk = total / (double)std::max(1, p.n_cu * kResidentPerCu);
    int heavy = 0;
    for (size_t k = 0; k < n - 1 && heavy < kMaxHeavy; ++k)
        if ((double)steps[k] > heavy_factor * bulk) ++heavy;
    // At most one generation of one-pixel waves (64 per heavy tile) in the
    // concurrent launch, shared by the launches in flight: past it the heavy
    // launch becomes the frame's critical path (the real FinalBaseMesh,
    // config 6: 196 tiles 0.686 ms, 87 tiles 0.666-0.684 ms; config 3's 79
    // tiles are under the cap).
    const int cap_waves = std::max(1, p.n_cu * kResidentPerCu * ctx->heavy_cap / 100 / std::max(1, concurrent));
    heavy = std::min(heavy, std::max(1, cap_waves / 64));
    // Heavy pixels (option heavy_pixels): the pixels whose own walk length
    // (their lockstep steps + 2 x the cooperative windows spent on them)
    // exceeds heavy_pixel_factor times the bulk estimate, most expensive
    // first, at most cap_waves of them.  A heavy tile holds a few dozen of its
    // 64 pixels over that bar (tools/heavy_pixel_model.py); splitting only
    // those keeps the rest of the tile in its lockstep wave.
    std::vector<unsigned> lane(n * 64);
    RT_HIP_CHECK(hipMemcpy(lane.data(), p.d_learn_lane, lane.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
    const double px_bar = ctx->heavy_pixel_factor / 100.0 * bulk;
    std::vector<int> hpix;
    for (size_t q = 0; q < n * 64; ++q)
        if ((double)lane[q] > px_bar) hpix.push_back((int)q);
    std::stable_sort(hpix.begin(), hpix.end(), [&](int x, int y) { return lane[x] > lane[y]; });
    if ((int)hpix.size() > cap_waves) hpix.resize(cap_waves);
    std::vector<unsigned long long> mask(n, 0ull);
    for (int q : hpix) mask[q >> 6] |= 1ull << (q & 63);
    if (std::getenv("RTAMD_DEBUG_ORDER")) {
        std::fprintf(stderr, "learn_order: %zu tiles, bulk estimate %.0f, %d heavy tiles, %zu heavy pixels; first:",
                     n, bulk, heavy, hpix.size());
        for (size_t k = 0; k < 6 && k < n; ++k) std::fprintf(stderr, " %d(%llu)", order[k], cost[order[k]]);
        std::fprintf(stderr, "\n");
    }
    if (p.orders.size() >= kMaxOrders) {
        // the oldest order may still steer a launch in flight on another stream
        RT_HIP_CHECK(hipDeviceSynchronize());
        poll_learning(p);
        free_order(p.orders.front());
        p.orders.erase(p.orders.begin());
    }
    PerDevice::Order o{p.learning_key, nullptr, n, heavy, nullptr, (int)hpix.size(), nullptr};
    hipError_t e = hipMalloc(&o.d_order, n * sizeof(int));
    if (e == hipSuccess) e = hipMemcpy(o.d_order, order.data(), n * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&o.d_mask, n * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemcpy(o.d_mask, mask.data(), n * sizeof(unsigned long long), hipMemcpyHostToDevice);
    if (e == hipSuccess && !hpix.empty()) e = hipMalloc(&o.d_hpix, hpix.size() * sizeof(int));
    if (e == hipSuccess && !hpix.empty())
        e = hipMemcpy(o.d_hpix, hpix.data(), hpix.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (o.d_order) free_order(o);
        RT_HIP_CHECK(e);
    }
    p.orders.push_back(std::move(o));
    return RT_OK;
}

// wave_tile -1: config 5 (112 MB of records, 4K) runs 16x4 tiles in 7.83-7.89
// ms per frame against 8.07-8.10 for 8x8; config 3 (6 MB, 1080p) runs 8x8 in
// 0.2942-0.2954 against 0.2965-0.2987 (profiles/r04/r4aa, r4ab).
// The records one ray walks: the reference's walk records, or one accel layout.
static size_t walk_bytes(const PerDevice& p) {
    return (size_t)(p.scene.n_layouts ? p.scene.layout_slots : p.scene.end2) * (p.scene.wide ? 64 : p.scene.half ? 16 : 32);
}

// The accel walk runs 16x4 tiles on every scene: config 3 0.1205-0.1212 ms per
// frame against 0.1226-0.1235 for 8x8, config 4 0.1482 against 0.1560-0.1569,
// config 6 0.1233-0.1239 against 0.1216-0.1222 (profiles/r05/r5ac).
static int wave_tile_of(const rt_ctx* ctx, const PerDevice& p) {
    if (ctx->wave_tile >= 0) return ctx->wave_tile;
    return (p.scene.n_layouts > 0 || walk_bytes(p) > kWin32Bytes) ? 1 : 0;
}

static int coop_window_of(const rt_ctx* ctx, const PerDevice& p) {
    if (ctx->coop_window) return ctx->coop_window;
    return walk_bytes(p) > kWin32Bytes ? 32 : 64;
}

static int set_schedule(const rt_ctx* ctx, PerDevice& p, TraceArgs& a, const rt_camera_ubo* cam,
                        const std::vector<int>* bands = nullptr) {
    a.wave_tile = wave_tile_of(ctx, p);
    // (the cooperative tail walks 32-B slots: not over half-format accel records)
    a.coop_lanes = (p.scene.half || p.scene.wide) ? 0 : ctx->coop_lanes >= 0 ? ctx->coop_lanes : (p.scene.n_layouts ? 0 : 1);
    a.walk = p.scene.n_layouts ? 2 : ctx->walk;          // accel: the walk-2 records only
    a.coop_walk = p.scene.n_layouts ? 0 : ctx->coop_walk;
    a.coop_win = coop_window_of(ctx, p);
    a.block_waves = ctx->block_waves;
    a.ext = ctx->ext;
    a.scene.spheres = p.d_spheres;
    a.scene.n_spheres = (a.ext & kExtSpheres) ? p.n_spheres : 0;
    a.scene.oct_mask = ctx->accel_octants;
    a.sky_enabled = cam->sky_enabled;
    a.frame_count = cam->frame_count;
    a.accum = nullptr;
    if (a.ext & kExtAccumulate) {
        if (a.n_frames != 1) {
            set_error("the accumulation extension renders one frame per launch (its sums are per pixel)");
            return RT_ERR_INVALID_ARG;
        }
        const size_t need = (size_t)a.tw * (size_t)a.th * 3;
        if (need != p.accum_n) {                 // a new frame partition starts from zero sums
            if (p.d_accum) {
                RT_HIP_CHECK(hipDeviceSynchronize());   // earlier frames in flight still add to the old sums
                (void)hipFree(p.d_accum);
            }
            p.d_accum = nullptr;
            p.accum_n = 0;
            RT_HIP_CHECK(hipMalloc(&p.d_accum, need * sizeof(float)));
            RT_HIP_CHECK(hipMemset(p.d_accum, 0, need * sizeof(float)));
            // hipMemset runs on the null stream, which the non-blocking launch
            // streams do not wait for: without this the zeroing could land on
            // sums frame 0 has already written (frames 1+ then differ, seen on a
            // second device of one context: tools/dbg/accum3.py, profiles/r04/r4g)
            RT_HIP_CHECK(hipDeviceSynchronize());
            p.accum_n = need;
        }
        a.accum = p.d_accum;
    }
    a.diag = nullptr;
    if (ctx->diag) {
        // 8 words per wave (+ 63 per heavy tile traced one pixel per wave)
        const int tw_w = 8 << a.wave_tile, th_w = 8 >> a.wave_tile;
        const int gw = std::max(4, a.block_waves);   // columns are rounded up to whole workgroups
        const size_t waves = (size_t)((a.tw + gw * tw_w - 1) / (gw * tw_w)) * ((a.th + th_w - 1) / th_w) * gw *
                             (size_t)a.n_frames;
        const size_t split = ctx->heavy_first ? (size_t)(ctx->heavy_tiles < 0 ? kMaxHeavy : ctx->heavy_tiles) * 63 : 0;
        const size_t words = (waves + split) * 8;
        if (words > p.diag_cap) {
            if (p.d_diag) {
                RT_HIP_CHECK(hipDeviceSynchronize());   // diagnostic launches in flight still write it
                (void)hipFree(p.d_diag);
            }
            p.d_diag = nullptr;
            p.diag_cap = 0;
            RT_HIP_CHECK(hipMalloc(&p.d_diag, words * sizeof(unsigned long long)));
            p.diag_cap = words;
        }
        p.diag_used = words;
        a.diag = p.d_diag;
    }
    return plan_order(ctx, p, a, cam, bands);
}

// Option graph: a plain kernel-0 launch (no counters, no diagnostics) is
// captured once per launch key into a HIP graph and replayed afterwards.  The
// key is every launch parameter the kernels read (scene, camera, frame
// geometry, schedule, learned order, heavy-tile count, outputs) plus the
// stream; the work counters, queue slots and the auxiliary stream / events a
// launch rotates through are not kernel inputs of the simple kernel.  In the
// captured graph the heavy-tile fork / join are edges, not events.
static std::vector<uint64_t> launch_key(const TraceArgs& a, hipStream_t s) {
    auto P = [](const void* q) { return (uint64_t)(uintptr_t)q; };
    auto F = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint64_t)u; };
    const DevScene& sc = a.scene;
    std::vector<uint64_t> k = {P(s), P(sc.nodes), P(sc.leafs), P(sc.pairs), P(sc.walk), P(sc.slot_node), P(sc.node_slot), P(sc.norms), P(sc.mats), P(sc.spheres),
            (uint64_t)sc.n_spheres, (uint64_t)sc.n_nodes, (uint64_t)sc.end, (uint64_t)sc.end2, (uint64_t)sc.n_tris,
            (uint64_t)sc.root_leaf, F(sc.root_box[0]), F(sc.root_box[1]), F(sc.root_box[2]), F(sc.root_box[3]),
            F(sc.root_box[4]), F(sc.root_box[5]), (uint64_t)a.n_frames, P(a.band_list), (uint64_t)a.list_stride,
            (uint64_t)a.width, (uint64_t)a.height, (uint64_t)a.max_bounces, (uint64_t)a.x0, (uint64_t)a.y0,
            (uint64_t)a.tw, (uint64_t)a.th, (uint64_t)a.band_h, (uint64_t)a.band_stride, (uint64_t)a.band_off,
            P(a.out_rgba), P(a.out_rad), (uint64_t)a.wave_tile,
            (uint64_t)a.coop_lanes, (uint64_t)a.ext, (uint64_t)a.sky_enabled,
            (uint64_t)a.frame_count, P(a.accum), (uint64_t)a.walk, (uint64_t)a.block_waves, P(a.tile_order),
            (uint64_t)a.heavy_tiles, (uint64_t)(a.aux_stream != nullptr), (uint64_t)a.heavy_fused, P(a.heavy_px),
            (uint64_t)a.n_heavy_px, P(a.tile_mask), (uint64_t)a.coop_walk, (uint64_t)a.coop_win,
            (uint64_t)a.split_bounce, P(a.q_slots), (uint64_t)a.q_waves, (uint64_t)a.q_grid};
    for (int f = 0; f < a.n_frames; ++f) {
        const CamF& c = a.cams[f];
        for (float v : {c.ox, c.oy, c.oz, c.lx, c.ly, c.lz, c.hx, c.hy, c.hz, c.vx, c.vy, c.vz}) k.push_back(F(v));
    }
    return k;
}

// Option split_bounce (accel walk, no extensions or counters): the stream's
// ray slots for a launch of tw x th x n_frames pixels.  Slots that must grow
// wait for the launches already on their stream, which may still use them.
static int attach_slots(const rt_ctx* ctx, PerDevice& p, TraceArgs& a, hipStream_t s) {
    a.q_slots = nullptr;
    a.split_bounce = 0;
    if (!p.scene.n_layouts || ctx->split_bounce <= 0 || ctx->split_bounce >= a.max_bounces || a.ext || a.diag ||
        a.counters)
        return RT_OK;
    // kernel 1's waves, as launch_trace lays out its grid (an upper bound)
    const int tw_w = 8 << a.wave_tile, th_w = 8 >> a.wave_tile, bw = std::max(1, a.block_waves);
    const long long waves = (long long)((a.tw + bw * tw_w - 1) / (bw * tw_w)) * bw *
                            ((a.th + th_w - 1) / th_w) * (long long)a.n_frames;
    // 3 KB of ray slots per wave (64 x 48 B): a one-frame 4K launch needs
    // ~400 MB.  Past kSplitSlotBytes the launch stays one kernel (advisor,
    // round 5: the slots only grow, per stream).
    if (waves > (1 << 24) || (size_t)waves * 64 * 48 > kSplitSlotBytes) return RT_OK;
    PerDevice::Slots* q = nullptr;
    for (auto& x : p.slots)
        if (x.s == s) { q = &x; break; }
    if (!q || q->waves < waves) {
        if (q) {
            RT_HIP_CHECK(hipStreamSynchronize(s));
            (void)hipFree(q->base);
            q->base = nullptr;
            q->waves = 0;
        } else {
            p.slots.push_back(PerDevice::Slots{s, nullptr, 0, 0});
            q = &p.slots.back();
        }
        size_t tb = 0;
        RT_HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, (const unsigned*)nullptr, (unsigned*)nullptr, 0u,
                                             (size_t)waves, rocprim::plus<unsigned>()));
        void* base = nullptr;
        const size_t bytes = (size_t)waves * 64 * 48 + 2 * ((size_t)waves * 4 + 256) + tb + 256;
        RT_HIP_CHECK(hipMalloc(&base, bytes));
        q->base = static_cast<char*>(base);
        q->waves = (int)waves;
        q->temp_bytes = tb;
    }
    a.split_bounce = ctx->split_bounce;
    a.q_slots = reinterpret_cast<float4*>(q->base);
    a.q_count = reinterpret_cast<unsigned*>(q->base + (size_t)q->waves * 64 * 48);
    a.q_prefix = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(a.q_count) + (size_t)q->waves * 4 + 256);
    a.q_temp = reinterpret_cast<char*>(a.q_prefix) + (size_t)q->waves * 4 + 256;
    a.q_temp_bytes = q->temp_bytes;
    a.q_waves = q->waves;
    a.q_grid = std::max(1, p.n_cu * 32);        // kernel 2: a full device of one-wave workgroups
    return RT_OK;
}

static int launch(const rt_ctx* ctx, PerDevice& p, const TraceArgs& a_in, hipStream_t s) {
    TraceArgs a = a_in;
    if (int rq = attach_slots(ctx, p, a, s)) return rq;
    // Only a frame of two launches (heavy tiles on an auxiliary stream,
    // heavy_stream 1) gains from a graph: its fork and join become edges.  A
    // single launch (the fused heavy tiles, or none) goes straight to the
    // stream: a graph launch adds ~9 us between frames (profiles/r02/graph).
    const bool plain = !a.counters && !a.diag;          // the production build (option "plain_kernels")
    int nk = 1;
    if (!ctx->graph || s == nullptr || a.counters || a.diag || !a.aux_stream) {
        RT_HIP_CHECK(launch_trace(a, s, &nk));
        if (plain) p.plain_kernels += (uint64_t)nk;
        return RT_OK;
    }
    std::vector<uint64_t> key = launch_key(a, s);
    for (auto& g : p.graphs)
        if (g.key == key) {
            RT_HIP_CHECK(hipGraphLaunch(g.exec, s));
            p.plain_kernels += g.kernels;
            return RT_OK;
        }
    hipGraph_t graph = nullptr;
    RT_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    const hipError_t le = launch_trace(a, s, &nk);
    const hipError_t ce = hipStreamEndCapture(s, &graph);
    if (le != hipSuccess || ce != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        set_error("graph capture: %s", hipGetErrorString(le != hipSuccess ? le : ce));
        return RT_ERR_HIP;
    }
    hipGraphExec_t exec = nullptr;
    const hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ie != hipSuccess) { set_error("graph instantiate: %s", hipGetErrorString(ie)); return RT_ERR_HIP; }
    if (p.graphs.size() >= kMaxGraphs) {          // replace the oldest-inserted entry
        const size_t k = p.graph_next++ % kMaxGraphs;
        (void)hipGraphExecDestroy(p.graphs[k].exec);
        p.graphs[k] = PerDevice::Graph{std::move(key), exec, nk};
    } else {
        p.graphs.push_back(PerDevice::Graph{std::move(key), exec, nk});
    }
    RT_HIP_CHECK(hipGraphLaunch(exec, s));
    p.plain_kernels += (uint64_t)nk;
    return RT_OK;
}

static CamF cam_from_ubo(const rt_camera_ubo* c) {
    CamF f;
    f.ox = c->origin[0];     f.oy = c->origin[1];     f.oz = c->origin[2];
    f.lx = c->lower_left[0]; f.ly = c->lower_left[1]; f.lz = c->lower_left[2];
    f.hx = c->horizontal[0]; f.hy = c->horizontal[1]; f.hz = c->horizontal[2];
    f.vx = c->vertical[0];   f.vy = c->vertical[1];   f.vz = c->vertical[2];
    return f;
}

extern "C" {

const char* rt_last_error(void) { return g_err; }

int rt_abi_version(size_t* stats_bytes, size_t* camera_bytes) {
    if (stats_bytes) *stats_bytes = sizeof(rt_stats);
    if (camera_bytes) *camera_bytes = sizeof(rt_camera_ubo);
    return RT_ABI_VERSION;
}

int rt_create(const int* device_ids, int n_devices, rt_ctx** out) {
    if (!out || n_devices < 1 || !device_ids) {
        set_error("rt_create: need out != NULL and n_devices >= 1 (there is no CPU backend)");
        return RT_ERR_INVALID_ARG;
    }
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        set_error("rt_create: no HIP device visible");
        return RT_ERR_NO_DEVICE;
    }
    rt_ctx* ctx = new (std::nothrow) rt_ctx;
    if (!ctx) { set_error("rt_create: out of memory"); return RT_ERR_OOM; }
    if (const char* v = std::getenv("RTAMD_WALK")) {
        const int w = std::atoi(v);
        ctx->walk = w == 0 ? 0 : 2;
    }
    // HIP reads GPU_MAX_HW_QUEUES once, when the runtime initialises (HIP's
    // default is 4 hardware queues per process); reported as option
    // "hw_queues" so a host can see whether its frames in flight get queues of
    // their own (rt_render_async's slots need async_slots + 2).
    if (const char* v = std::getenv("GPU_MAX_HW_QUEUES")) {
        const int q = std::atoi(v);
        if (q > 0) ctx->hw_queues = q;
    }
    if (const char* v = std::getenv("RTAMD_COOP_WALK")) ctx->coop_walk = std::atoi(v) ? 1 : 0;
    if (const char* v = std::getenv("RTAMD_ACCEL")) {
        const int k = std::atoi(v);
        ctx->accel = k == 1 || k == 8 ? k : 0;
    }
    if (const char* v = std::getenv("RTAMD_ACCEL_HALF")) ctx->accel_half = std::atoi(v) ? 1 : 0;
    if (const char* v = std::getenv("RTAMD_ACCEL_WIDE")) ctx->accel_wide = std::atoi(v) ? 1 : 0;
    if (const char* v = std::getenv("RTAMD_HEAVY_FIRST")) ctx->heavy_first = std::atoi(v) ? 1 : 0;
    if (const char* v = std::getenv("RTAMD_XCD_ORDER")) ctx->xcd_order = std::max(0, std::min(4096, std::atoi(v)));
    if (const char* v = std::getenv("RTAMD_ACCEL_OCTANTS")) ctx->accel_octants = std::atoi(v) & 7;
    if (const char* v = std::getenv("RTAMD_HEAVY_TILES")) ctx->heavy_tiles = std::max(-1, std::atoi(v));
    if (const char* v = std::getenv("RTAMD_LEARN_COST")) ctx->learn_cost = std::atoi(v) ? 1 : 0;
    if (const char* v = std::getenv("RTAMD_ORDER_SPLIT")) ctx->order_split = std::max(0, std::min(100, std::atoi(v)));
    if (const char* v = std::getenv("RTAMD_HEAVY_FACTOR")) ctx->heavy_factor = std::max(10, std::atoi(v));
    if (const char* v = std::getenv("RTAMD_HEAVY_STREAM")) ctx->heavy_stream = std::max(0, std::min(2, std::atoi(v)));
    if (const char* v = std::getenv("RTAMD_HEAVY_PIXELS")) ctx->heavy_pixels = std::atoi(v) ? 1 : 0;
    if (const char* v = std::getenv("RTAMD_GRAPH")) ctx->graph = std::atoi(v) ? 1 : 0;
    if (const char* v = std::getenv("RTAMD_BLOCK_WAVES")) {
        const int bw = std::atoi(v);
        ctx->block_waves = bw == 1 ? 1 : 4;
    }
    if (const char* v = std::getenv("RTAMD_COOP_LANES")) ctx->coop_lanes = std::max(-1, std::min(64, std::atoi(v)));
    // RTAMD_OPTS="name=value,...": any rt_set_option defaults (A/B runs)
    if (const char* v = std::getenv("RTAMD_OPTS")) {
        std::string all(v);
        size_t pos = 0;
        while (pos < all.size()) {
            size_t comma = all.find(',', pos);
            if (comma == std::string::npos) comma = all.size();
            const std::string item = all.substr(pos, comma - pos);
            const size_t eq = item.find('=');
            if (eq != std::string::npos &&
                rt_set_option(ctx, item.substr(0, eq).c_str(), std::atoll(item.c_str() + eq + 1)) != RT_OK) {
                rt_destroy(ctx);
                return RT_ERR_INVALID_ARG;       // rt_set_option's message names the option
            }
            pos = comma + 1;
        }
    }
    for (int k = 0; k < n_devices; ++k) {
        const int d = device_ids[k];
        if (d < 0 || d >= count) {
            set_error("rt_create: device id %d out of range (0..%d)", d, count - 1);
            rt_destroy(ctx);
            return RT_ERR_NO_DEVICE;
        }
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            set_error("rt_create: device %d is not gfx950 (%s)", d, prop.gcnArchName);
            rt_destroy(ctx);
            return RT_ERR_NO_DEVICE;
        }
        PerDevice p;
        p.device = d;
        hipError_t e = hipSetDevice(d);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreate(&p.ev0);
        if (e == hipSuccess) e = hipEventCreate(&p.ev1);
        if (e == hipSuccess) e = hipMalloc(&p.d_counters, sizeof(Counters));
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&p.copy_stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&p.copy_stream2, hipStreamNonBlocking);
        for (int k2 = 0; k2 < kMaxSlots && e == hipSuccess; ++k2) {
            e = hipEventCreateWithFlags(&p.traced[k2], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&p.copied[k2], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&p.copied2[k2], hipEventDisableTiming);
        }
        p.n_cu = prop.multiProcessorCount;
        ctx->dev.push_back(p);
        if (e != hipSuccess) {
            set_error("rt_create: HIP setup on device %d failed: %s", d, hipGetErrorString(e));
            rt_destroy(ctx);
            return RT_ERR_HIP;
        }
    }
    *out = ctx;
    return RT_OK;
}

int rt_destroy(rt_ctx* ctx) {
    if (!ctx) return RT_OK;
    for (PerDevice& p : ctx->dev) {
        (void)hipSetDevice(p.device);
        if (p.stream) (void)hipStreamSynchronize(p.stream);
        if (p.copy_stream) (void)hipStreamSynchronize(p.copy_stream);
        if (p.copy_stream2) (void)hipStreamSynchronize(p.copy_stream2);
        free_scene(p);
        for (int k2 = 0; k2 < kMaxSlots; ++k2) {
            if (p.slot_stream[k2]) (void)hipStreamSynchronize(p.slot_stream[k2]);
            if (p.d_ring[k2]) (void)hipFree(p.d_ring[k2]);
            if (p.traced[k2]) (void)hipEventDestroy(p.traced[k2]);
            if (p.copied[k2]) (void)hipEventDestroy(p.copied[k2]);
            if (p.copied2[k2]) (void)hipEventDestroy(p.copied2[k2]);
            if (p.slot_stream[k2]) (void)hipStreamDestroy(p.slot_stream[k2]);
        }
        if (p.copy_stream) (void)hipStreamDestroy(p.copy_stream);
        if (p.copy_stream2) (void)hipStreamDestroy(p.copy_stream2);
        if (p.d_counters) (void)hipFree(p.d_counters);
        if (p.d_diag) (void)hipFree(p.d_diag);
        if (p.d_learn) (void)hipFree(p.d_learn);
        if (p.d_learn_lane) (void)hipFree(p.d_learn_lane);
        if (p.d_learn_scratch) (void)hipFree(p.d_learn_scratch);
        if (p.h_nhpix) (void)hipHostFree(p.h_nhpix);
        if (p.learn_ev) (void)hipEventDestroy(p.learn_ev);
        free_orders(p);
        free_graphs(p);
        for (auto& l : p.band_lists) (void)hipFree(l.d);
        p.band_lists.clear();
        for (int k = 0; k < 4; ++k) {
            if (p.aux[k]) (void)hipStreamDestroy(p.aux[k]);
            if (p.aux_fork[k]) (void)hipEventDestroy(p.aux_fork[k]);
            if (p.aux_join[k]) (void)hipEventDestroy(p.aux_join[k]);
        }
        for (auto& q : p.slots) (void)hipFree(q.base);
        p.slots.clear();
        if (p.d_accum) (void)hipFree(p.d_accum);
        if (p.d_spheres) (void)hipFree(p.d_spheres);
        if (p.d_rgba) (void)hipFree(p.d_rgba);
        if (p.d_rad) (void)hipFree(p.d_rad);
        if (p.ev0) (void)hipEventDestroy(p.ev0);
        if (p.ev1) (void)hipEventDestroy(p.ev1);
        if (p.stream) (void)hipStreamDestroy(p.stream);
    }
    delete ctx;
    return RT_OK;
}

int rt_upload_scene(rt_ctx* ctx, const void* vertices, size_t vertex_bytes,
                    const void* materials, size_t material_bytes,
                    const void* bvh_nodes, size_t bvh_bytes) {
    if (!ctx) { set_error("rt_upload_scene: null context"); return RT_ERR_INVALID_ARG; }
    HostScene hs;
    const char* err = nullptr;
    int rc = build_host_scene(vertices, vertex_bytes, materials, material_bytes,
                              bvh_nodes, bvh_bytes, &hs, &err);
    if (rc != RT_OK) { set_error("rt_upload_scene: %s", err); return rc; }
    // walk 2's records (DevScene::walk; rt_internal.h): the reference's
    // preorder with every leaf's triangle inlined after its box, so an
    // internal node takes one 32-B slot and a leaf two.  slot(i) = i + the
    // leaves before i; an internal node's left child is the next slot, a
    // leaf's successor (its skip, i+1) the slot after its two, and only the
    // internal skip is stored, as a slot.  The visit sequence is the
    // reference's, node for node.
    // Option leaf_align: a leaf that would start in the last slot of a 128-B
    // line (and straddle two) starts one slot later; its predecessor's pad bit
    // (a leaf's bit 29 of word [0].w, an internal node's bit 2 of word [1].w)
    // tells the walk to step over the pad slot.
    // Only the root's subtree, [0, end): nodes past the root's skip are
    // never visited by the reference's DFS (compute_dynamic_ray.comp:185-210).
    const size_t n2 = (size_t)hs.end;
    std::vector<int> slot(n2 + 1);
    std::vector<uint8_t> padded(n2 + 1, 0);       // a pad slot precedes node i
    size_t n_leaves = 0;
    for (size_t i = 0; i < n2; ++i) {
        uint32_t fl;
        std::memcpy(&fl, &hs.nodes[2 * i + 1].w, 4);
        n_leaves += (fl & 2u) ? 1 : 0;
    }
    const bool align = ctx->leaf_align == 1 || (ctx->leaf_align == 2 && (n2 + n_leaves) * 32 > kWin32Bytes);
    size_t nslot = 0, n_pads = 0;
    for (size_t i = 0; i < n2; ++i) {
        uint32_t fl;
        std::memcpy(&fl, &hs.nodes[2 * i + 1].w, 4);
        if (align && (fl & 2u) && nslot % 4 == 3) {
            padded[i] = 1;
            ++nslot;
            ++n_pads;
        }
        slot[i] = (int)nslot;
        nslot += (fl & 2u) ? 2 : 1;
        if (nslot >= kMaxWalkSlots) {
            free_host_scene(&hs);
            set_error("rt_upload_scene: %zu nodes: at most %u walk slots (4 GB of walk records) supported", n2,
                      kMaxWalkSlots);
            return RT_ERR_BAD_SCENE;
        }
    }
    slot[n2] = (int)nslot;
    std::vector<float4> walk(2 * nslot + 4, make_float4(0.f, 0.f, 0.f, 0.f));   // + padding read at the end
    std::vector<int> slot_node(nslot + 1, -1);
    for (size_t i = 0; i < n2; ++i) {
        const size_t w = 2 * (size_t)slot[i];
        slot_node[slot[i]] = (int)i;
        walk[w] = hs.nodes[2 * i];
        walk[w + 1] = hs.nodes[2 * i + 1];
        uint32_t fl, link;
        std::memcpy(&fl, &hs.nodes[2 * i + 1].w, 4);
        std::memcpy(&link, &hs.nodes[2 * i].w, 4);
        if (!(fl & 2u)) {                                   // internal: the skip as a slot (< 2^30: bit 30 clear)
            const uint32_t sk = link & 0x7FFFFFFFu;
            const uint32_t w0 = (uint32_t)slot[sk] | (link & 0x80000000u);
            std::memcpy(&walk[w].w, &w0, 4);
            if (padded[i + 1]) {                            // the left child (i+1) sits past a pad slot
                uint32_t w1;
                std::memcpy(&w1, &walk[w + 1].w, 4);
                w1 |= 4u;
                std::memcpy(&walk[w + 1].w, &w1, 4);
            }
            continue;
        }
        uint32_t tri;
        std::memcpy(&tri, &hs.leafs[3 * i].w, 4);
        if ((link & 0x7FFFFFFFu) != i + 1 || tri >= (1u << 29)) {
            free_host_scene(&hs);
            set_error("rt_upload_scene: leaf %zu: skip %u is not i+1 or triangle index %u too large", i,
                      link & 0x7FFFFFFFu, tri);
            return RT_ERR_BAD_SCENE;
        }
        const uint32_t w0 = tri | (padded[i + 1] ? 1u << 29 : 0u) | (1u << 30) | (link & 0x80000000u);
        std::memcpy(&walk[w].w, &w0, 4);
        walk[w + 1].w = hs.leafs[3 * i].x;                                   // v0.x
        const float4 P0 = hs.leafs[3 * i], P1 = hs.leafs[3 * i + 1], P2 = hs.leafs[3 * i + 2];
        walk[w + 2] = make_float4(P0.y, P0.z, P1.x, P1.y);                   // v0.yz, e1.xy
        walk[w + 3] = make_float4(P1.z, P2.x, P2.y, P2.z);                   // e1.z, e2
    }
    // Option accel: the binned-SAH records (accel_build.h), built once for
    // every device; the reference's walk records above stay beside them for
    // the fallback, and the node-indexed arrays (walk 0, the frontier walk of
    // heavy pixels) are not needed.
    // Past the slot cap 8 layouts become 1, and a scene too large for one
    // walks the reference's own tree (accel_used says which: 8, 1 or 0).
    AccelHost ah;
    bool acc = false;
    if (ctx->accel) {
        std::string msg;
        const int rc = accel_build_fit(vertices, vertex_bytes, materials, material_bytes, bvh_nodes,
                                       (size_t)hs.end * RT_NODE_RECORD_BYTES, ctx->accel, &ah, &msg,
                                       ctx->accel_wide ? 2 : ctx->accel_half ? 1 : 0, accel_cap_slots());
        if (rc != 0 && rc != kAccelTooBig) {
            free_host_scene(&hs);
            set_error("rt_upload_scene: %s", msg.c_str());
            return RT_ERR_BAD_SCENE;
        }
        acc = rc == 0;
    }
    ctx->has_scene = false;
    for (PerDevice& p : ctx->dev) {
        RT_HIP_CHECK(hipSetDevice(p.device));
        // Like vkDeviceWaitIdle (VulkanEngine.java:321): every launch and copy
        // still in flight on this device (rt_render_async's slot and copy
        // streams, a caller's streams of the *_device calls, the heavy-tile
        // streams) may read the old scene, so the whole device drains before
        // its buffers are freed.
        RT_HIP_CHECK(hipDeviceSynchronize());
        free_scene(p);
        DevScene s;
        s.n_nodes = hs.n_nodes;
        s.end = hs.end;
        s.n_tris = hs.n_tris;
        s.root_leaf = hs.root_leaf;
        std::memcpy(s.root_box, hs.root_box, sizeof s.root_box);
        // nodes and leafs are padded by one record: walks read the record at
        // index end (the node after the last) before they test for the end.
        const size_t nn = (size_t)hs.n_nodes;
        const size_t nb = sizeof(float4) * (2 * nn + 2);
        const size_t lb = sizeof(float4) * (3 * nn + 1);
        const size_t pb = sizeof(float4) * 4 * (size_t)(hs.n_nodes ? hs.n_nodes : 1);
        const size_t mb = sizeof(float4) * (size_t)(hs.n_tris ? hs.n_tris : 1);
        hipError_t e = hipSuccess;
        if (acc) {
            s.n_layouts = ah.n_layouts;
            s.layout_slots = ah.slots;
            s.half = ah.format == 1 ? 1 : 0;
            s.wide = ah.format == 2 ? 1 : 0;
            s.relax_half = ah.relax_max;
            s.root_enter = ah.format == 0 && !ah.root_leaf && ah.slots > 1 ? 1 : 0;
            s.root_first_leaf = 0;
            if (s.root_enter)
                for (int o = 0; o < ah.n_layouts; ++o)
                    s.root_first_leaf |= (int)(ah.rec[8 * (size_t)o * (size_t)ah.slots + 7] >> 31) << o;
            s.end = ah.slots;
            s.end2 = ah.n_layouts * ah.slots;
            s.root_leaf = ah.root_leaf;
            s.end2_ref = (int)nslot;
            s.ref_padded = n_pads > 0 ? 1 : 0;
            e = hipMalloc(&s.walk, ah.rec.size() * sizeof(uint32_t));
            if (e == hipSuccess) e = hipMalloc(&s.walk_ref, walk.size() * sizeof(float4));
            if (e == hipSuccess)
                e = hipMemcpy(s.walk, ah.rec.data(), ah.rec.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
            if (e == hipSuccess)
                e = hipMemcpy(s.walk_ref, walk.data(), walk.size() * sizeof(float4), hipMemcpyHostToDevice);
        } else {
            e = hipMalloc(&s.nodes, nb);
            if (e == hipSuccess) e = hipMalloc(&s.leafs, lb);
            if (e == hipSuccess) e = hipMalloc(&s.pairs, pb);
            if (e == hipSuccess) e = hipMemset(s.nodes + 2 * nn, 0, 2 * sizeof(float4));
            if (e == hipSuccess) e = hipMemset(s.leafs + 3 * nn, 0, sizeof(float4));
            s.end2 = (int)nslot;
            s.padded = n_pads > 0 ? 1 : 0;
            if (e == hipSuccess) e = hipMalloc(&s.walk, walk.size() * sizeof(float4));
            if (e == hipSuccess) e = hipMalloc(&s.slot_node, slot_node.size() * sizeof(int));
            if (e == hipSuccess) e = hipMalloc(&s.node_slot, slot.size() * sizeof(int));
            if (e == hipSuccess)
                e = hipMemcpy(s.node_slot, slot.data(), slot.size() * sizeof(int), hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(s.walk, walk.data(), walk.size() * sizeof(float4), hipMemcpyHostToDevice);
            if (e == hipSuccess)
                e = hipMemcpy(s.slot_node, slot_node.data(), slot_node.size() * sizeof(int), hipMemcpyHostToDevice);
            if (e == hipSuccess && hs.n_nodes)
                e = hipMemcpy(s.nodes, hs.nodes, nb - 2 * sizeof(float4), hipMemcpyHostToDevice);
            if (e == hipSuccess && hs.n_nodes)
                e = hipMemcpy(s.leafs, hs.leafs, lb - sizeof(float4), hipMemcpyHostToDevice);
            if (e == hipSuccess && hs.n_nodes) e = hipMemcpy(s.pairs, hs.pairs, pb, hipMemcpyHostToDevice);
        }
        if (e == hipSuccess) e = hipMalloc(&s.norms, kShadeStride * mb);
        if (e == hipSuccess) s.mats = s.norms + 1;
        if (e == hipSuccess && hs.n_tris)
            e = hipMemcpy2D(s.norms, kShadeStride * sizeof(float4), hs.norms, sizeof(float4), sizeof(float4),
                            (size_t)hs.n_tris, hipMemcpyHostToDevice);
        if (e == hipSuccess && hs.n_tris)
            e = hipMemcpy2D(s.mats, kShadeStride * sizeof(float4), hs.mats, sizeof(float4), sizeof(float4),
                            (size_t)hs.n_tris, hipMemcpyHostToDevice);
        // the padding memsets ran on the null stream: complete before any
        // launch stream (non-blocking) reads the scene
        if (e == hipSuccess) e = hipDeviceSynchronize();
        p.scene = s;
        if (e != hipSuccess) {
            set_error("rt_upload_scene: device %d: %s", p.device, hipGetErrorString(e));
            free_scene(p);
            free_host_scene(&hs);
            return e == hipErrorOutOfMemory ? RT_ERR_OOM : RT_ERR_HIP;
        }
    }
    ctx->n_nodes = hs.n_nodes;
    ctx->n_tris = hs.n_tris;
    ctx->max_depth = hs.max_depth;
    ctx->has_scene = true;
    ++ctx->scene_gen;
    free_host_scene(&hs);
    return RT_OK;
}

int rt_upload_spheres(rt_ctx* ctx, const float* spheres, int n_spheres) {
    if (!ctx) { set_error("rt_upload_spheres: null context"); return RT_ERR_INVALID_ARG; }
    if (n_spheres < 0 || n_spheres > 65536 || (n_spheres > 0 && !spheres)) {
        set_error("rt_upload_spheres: need 0 <= n_spheres <= 65536 and a buffer of 8 floats per sphere");
        return RT_ERR_INVALID_ARG;
    }
    for (int k = 0; k < n_spheres; ++k) {
        const float* s = spheres + 8 * (size_t)k;
        if (!std::isfinite(s[0]) || !std::isfinite(s[1]) || !std::isfinite(s[2]) || !std::isfinite(s[3]) ||
            !(s[3] > 0.0f)) {
            set_error("rt_upload_spheres: sphere %d: centre must be finite and radius finite and > 0", k);
            return RT_ERR_INVALID_ARG;
        }
    }
    for (PerDevice& p : ctx->dev) {
        RT_HIP_CHECK(hipSetDevice(p.device));
        RT_HIP_CHECK(hipDeviceSynchronize());            // frames in flight may read the old spheres
        if (p.d_spheres) (void)hipFree(p.d_spheres);
        p.d_spheres = nullptr;
        p.n_spheres = 0;
        if (n_spheres == 0) continue;
        const size_t bytes = sizeof(float) * 8 * (size_t)n_spheres;
        hipError_t e = hipMalloc(&p.d_spheres, bytes);
        if (e == hipSuccess) e = hipMemcpy(p.d_spheres, spheres, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            set_error("rt_upload_spheres: device %d: %s", p.device, hipGetErrorString(e));
            if (p.d_spheres) (void)hipFree(p.d_spheres);
            p.d_spheres = nullptr;
            return e == hipErrorOutOfMemory ? RT_ERR_OOM : RT_ERR_HIP;
        }
        p.n_spheres = n_spheres;
    }
    ++ctx->scene_gen;    // learned tile orders see the new work
    return RT_OK;
}

int rt_scene_info(rt_ctx* ctx, size_t* n_nodes, size_t* n_tris, int* max_depth) {
    if (!ctx) { set_error("rt_scene_info: null context"); return RT_ERR_INVALID_ARG; }
    if (!ctx->has_scene) { set_error("rt_scene_info: no scene uploaded"); return RT_ERR_NO_SCENE; }
    if (n_nodes) *n_nodes = (size_t)ctx->n_nodes;
    if (n_tris) *n_tris = (size_t)ctx->n_tris;
    if (max_depth) *max_depth = ctx->max_depth;
    return RT_OK;
}

static int check_render_args(rt_ctx* ctx, const rt_camera_ubo* cam, int width, int height,
                             int max_bounces, const char* fn) {
    if (!ctx || !cam) { set_error("%s: null context or camera", fn); return RT_ERR_INVALID_ARG; }
    if (width < 1 || height < 1 || (int64_t)width * (int64_t)height > (int64_t)1 << 31) {
        set_error("%s: bad frame size %dx%d", fn, width, height);
        return RT_ERR_INVALID_ARG;
    }
    if (max_bounces < 1 || max_bounces > 1024) {
        set_error("%s: max_bounces must be in [1, 1024], got %d", fn, max_bounces);
        return RT_ERR_INVALID_ARG;
    }
    if (!ctx->has_scene) { set_error("%s: no scene uploaded", fn); return RT_ERR_NO_SCENE; }
    return RT_OK;
}

static int ensure_out(PerDevice& p, size_t pixels, bool rad) {
    if (pixels > p.out_cap || (rad && !p.d_rad)) {
        if (p.d_rgba) (void)hipFree(p.d_rgba);
        if (p.d_rad) (void)hipFree(p.d_rad);
        p.d_rgba = nullptr;
        p.d_rad = nullptr;
        p.out_cap = 0;
        RT_HIP_CHECK(hipMalloc(&p.d_rgba, pixels * 4));
        if (rad) RT_HIP_CHECK(hipMalloc(&p.d_rad, pixels * 12));
        p.out_cap = pixels;
    }
    return RT_OK;
}

static int collect_stats(const rt_ctx* ctx, PerDevice& p, uint64_t pixels, rt_stats* stats, bool accumulate);

int rt_render_tile_device(rt_ctx* ctx, const rt_camera_ubo* cam, int width, int height,
                          int max_bounces, int x0, int y0, int tile_w, int tile_h,
                          void* d_out_rgba, void* d_out_radiance, void* stream, rt_stats* stats) {
    int rc = check_render_args(ctx, cam, width, height, max_bounces, "rt_render_tile_device");
    if (rc) return rc;
    if (tile_w < 1 || tile_h < 1 || x0 < 0 || y0 < 0 || x0 + tile_w > width || y0 + tile_h > height) {
        set_error("rt_render_tile_device: tile (%d,%d %dx%d) outside the %dx%d frame",
                  x0, y0, tile_w, tile_h, width, height);
        return RT_ERR_INVALID_ARG;
    }
    PerDevice& p = ctx->dev[0];
    RT_HIP_CHECK(hipSetDevice(p.device));
    hipStream_t s = static_cast<hipStream_t>(stream);   // NULL = the null stream
    TraceArgs a;
    a.scene = p.scene;
    a.cams[0] = cam_from_ubo(cam);
    a.n_frames = 1;
    a.width = width; a.height = height; a.max_bounces = max_bounces;
    a.x0 = x0; a.y0 = y0; a.tw = tile_w; a.th = tile_h;
    a.band_h = tile_h; a.band_stride = 1; a.band_off = 0;
    a.band_list = nullptr;
    a.list_stride = 0;
    a.out_rgba = static_cast<uchar4*>(d_out_rgba);
    a.out_rad = static_cast<float*>(d_out_radiance);
    // counters before set_schedule: a counting launch must not become the
    // (non-counting) learning launch of the heavy-first order
    a.counters = stats ? p.d_counters : nullptr;
    if (int rs = set_schedule(ctx, p, a, cam)) return rs;
    if (stats) {
        RT_HIP_CHECK(hipMemsetAsync(p.d_counters, 0, sizeof(Counters), s));
        RT_HIP_CHECK(hipEventRecord(p.ev0, s));
    }
    if (int rl = launch(ctx, p, a, s)) return rl;
    if (int ro = learn_order(ctx, p, a, s)) return ro;
    if (stats) {
        RT_HIP_CHECK(hipEventRecord(p.ev1, s));
        RT_HIP_CHECK(hipEventSynchronize(p.ev1));
        return collect_stats(ctx, p, (uint64_t)tile_w * (uint64_t)tile_h, stats, false);
    }
    return RT_OK;
}

int rt_band_rows(int height, int band_h, int band_stride, int band_off) {
    if (height < 1 || band_h < 1 || band_stride < 1 || band_off < 0 || band_off >= band_stride) return -1;
    // rows of frame [0, height) whose band index b = row / band_h has b % band_stride == band_off
    const int n_bands = (height + band_h - 1) / band_h;
    int rows = 0;
    for (int b = band_off; b < n_bands; b += band_stride)
        rows += std::min(band_h, height - b * band_h);
    return rows;
}

// A band list on the device (rt_render_batch_device), uploaded once per
// distinct list and kept for the context's lifetime (a launch in flight may
// still read it); past kMaxBandLists the device is drained and they are
// dropped.
static constexpr size_t kMaxBandLists = 256;

static int device_band_list(PerDevice& p, const std::vector<int>& bands, const int** out) {
    for (const auto& l : p.band_lists)
        if (l.bands == bands) { *out = l.d; return RT_OK; }
    if (p.band_lists.size() >= kMaxBandLists) {
        RT_HIP_CHECK(hipDeviceSynchronize());
        for (auto& l : p.band_lists) (void)hipFree(l.d);
        p.band_lists.clear();
    }
    int* d = nullptr;
    RT_HIP_CHECK(hipMalloc(&d, std::max<size_t>(1, bands.size()) * sizeof(int)));
    const hipError_t e = hipMemcpy(d, bands.data(), bands.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        RT_HIP_CHECK(e);
    }
    p.band_lists.push_back(PerDevice::BandList{bands, d});
    *out = d;
    return RT_OK;
}

// One launch over the same rows of n_frames frames (camera cams[f] each):
// the band_h-row bands b with b mod band_stride == band_off, or, with
// `bands`, the listed bands; rows per frame = rows.  Outputs hold the frames
// one after another (n_frames x rows x width).
static int render_rows_on(const rt_ctx* ctx, PerDevice& p, const rt_camera_ubo* cams, int n_frames, int width,
                          int height, int max_bounces, int band_h, int band_stride, int band_off,
                          const std::vector<int>* bands, int rows, uchar4* d_rgba, float* d_rad, hipStream_t s,
                          bool count, int list_stride = 0, int x0 = 0, int y0 = 0, int tile_w = 0,
                          bool row_offsets = false) {
    TraceArgs a;
    a.scene = p.scene;
    for (int f = 0; f < n_frames; ++f) a.cams[f] = cam_from_ubo(cams + f);
    a.n_frames = n_frames;
    a.width = width; a.height = height; a.max_bounces = max_bounces;
    a.x0 = x0; a.y0 = y0; a.tw = tile_w > 0 ? tile_w : width; a.th = rows;
    a.band_h = band_h; a.band_stride = band_stride; a.band_off = band_off;
    a.band_list = nullptr;
    a.list_stride = bands ? list_stride : 0;
    if (bands)
        if (int rb = device_band_list(p, *bands, &a.band_list)) return rb;
    // row_offsets: the list ends with each frame's first output row
    a.row_off = (bands && row_offsets) ? a.band_list + (size_t)n_frames * list_stride : nullptr;
    a.out_rgba = d_rgba;
    a.out_rad = d_rad;
    a.counters = count ? p.d_counters : nullptr;
    if (int rs = set_schedule(ctx, p, a, cams, bands)) return rs;
    if (count) {
        RT_HIP_CHECK(hipMemsetAsync(p.d_counters, 0, sizeof(Counters), s));
        RT_HIP_CHECK(hipEventRecord(p.ev0, s));   // the timing events exist for stats only
    }
    if (int rl = launch(ctx, p, a, s)) return rl;
    if (int ro = learn_order(ctx, p, a, s)) return ro;
    if (count) RT_HIP_CHECK(hipEventRecord(p.ev1, s));
    return RT_OK;
}

static int render_bands_on(const rt_ctx* ctx, PerDevice& p, const rt_camera_ubo* cam, int width, int height,
                           int max_bounces, int band_h, int band_stride, int band_off, int rows,
                           uchar4* d_rgba, float* d_rad, hipStream_t s, bool count) {
    return render_rows_on(ctx, p, cam, 1, width, height, max_bounces, band_h, band_stride, band_off, nullptr, rows,
                          d_rgba, d_rad, s, count);
}

static int collect_stats(const rt_ctx* ctx, PerDevice& p, uint64_t pixels, rt_stats* stats, bool accumulate) {
    (void)ctx;
    Counters c;
    RT_HIP_CHECK(hipMemcpy(&c, p.d_counters, sizeof c, hipMemcpyDeviceToHost));
    float ms = 0.f;
    RT_HIP_CHECK(hipEventElapsedTime(&ms, p.ev0, p.ev1));
    if (!accumulate) std::memset(stats, 0, sizeof *stats);
    stats->pixels += pixels;
    stats->segments += c.segments;
    stats->node_visits += c.node_visits;
    stats->tri_tests += c.tri_tests;
    stats->mat_reads += c.mat_reads;
    if (ms > stats->ms) stats->ms = ms;
    return RT_OK;
}

int rt_render_bands_device(rt_ctx* ctx, const rt_camera_ubo* cam, int width, int height, int max_bounces,
                           int band_h, int band_stride, int band_off,
                           void* d_out_rgba, void* d_out_radiance, void* stream, rt_stats* stats) {
    int rc = check_render_args(ctx, cam, width, height, max_bounces, "rt_render_bands_device");
    if (rc) return rc;
    const int rows = rt_band_rows(height, band_h, band_stride, band_off);
    if (rows < 0) {
        set_error("rt_render_bands_device: bad bands (band_h %d, stride %d, offset %d)", band_h, band_stride, band_off);
        return RT_ERR_INVALID_ARG;
    }
    if (rows == 0) {
        if (stats) std::memset(stats, 0, sizeof *stats);
        return RT_OK;
    }
    PerDevice& p = ctx->dev[0];
    RT_HIP_CHECK(hipSetDevice(p.device));
    hipStream_t s = static_cast<hipStream_t>(stream);   // NULL = the null stream
    rc = render_bands_on(ctx, p, cam, width, height, max_bounces, band_h, band_stride, band_off, rows,
                         static_cast<uchar4*>(d_out_rgba), static_cast<float*>(d_out_radiance), s, stats != nullptr);
    if (rc) return rc;
    if (stats) {
        RT_HIP_CHECK(hipEventSynchronize(p.ev1));
        return collect_stats(ctx, p, (uint64_t)rows * width, stats, false);
    }
    return RT_OK;
}

int rt_band_list_rows(int height, int band_h, const int32_t* bands, int n_bands) {
    if (height < 1 || band_h < 1 || n_bands < 0 || (n_bands > 0 && !bands)) return -1;
    const int n_all = (height + band_h - 1) / band_h;
    int rows = 0;
    for (int k = 0; k < n_bands; ++k) {
        if (bands[k] < 0 || bands[k] >= n_all || (k > 0 && bands[k] <= bands[k - 1])) return -1;
        rows += std::min(band_h, height - bands[k] * band_h);
    }
    return rows;
}

int rt_render_batch_device(rt_ctx* ctx, const rt_camera_ubo* cams, int n_frames, int width, int height,
                           int max_bounces, int band_h, const int32_t* bands, int n_bands,
                           void* d_out_rgba, void* d_out_radiance, void* stream, rt_stats* stats) {
    int rc = check_render_args(ctx, cams, width, height, max_bounces, "rt_render_batch_device");
    if (rc) return rc;
    if (n_frames < 1 || n_frames > kMaxBatch) {
        set_error("rt_render_batch_device: n_frames must be in [1, %d], got %d", kMaxBatch, n_frames);
        return RT_ERR_INVALID_ARG;
    }
    int rows;
    std::vector<int> list;
    if (bands) {
        rows = rt_band_list_rows(height, band_h, bands, n_bands);
        if (rows < 0) {
            set_error("rt_render_batch_device: bad band list (band_h %d, %d bands: indices must increase and lie "
                      "below ceil(height / band_h))", band_h, n_bands);
            return RT_ERR_INVALID_ARG;
        }
        list.assign(bands, bands + n_bands);
    } else {
        band_h = height;                     // the whole frame
        rows = height;
    }
    if (rows == 0) {
        if (stats) std::memset(stats, 0, sizeof *stats);
        return RT_OK;
    }
    PerDevice& p = ctx->dev[0];
    RT_HIP_CHECK(hipSetDevice(p.device));
    hipStream_t s = static_cast<hipStream_t>(stream);   // NULL = the null stream
    rc = render_rows_on(ctx, p, cams, n_frames, width, height, max_bounces, band_h, 1, 0, bands ? &list : nullptr,
                        rows, static_cast<uchar4*>(d_out_rgba), static_cast<float*>(d_out_radiance), s,
                        stats != nullptr);
    if (rc) return rc;
    if (stats) {
        RT_HIP_CHECK(hipEventSynchronize(p.ev1));
        return collect_stats(ctx, p, (uint64_t)rows * width * n_frames, stats, false);
    }
    return RT_OK;
}

int rt_render_batch_rect_device(rt_ctx* ctx, const rt_camera_ubo* cams, int n_frames, int width, int height,
                                int max_bounces, int x0, int y0, int tile_w, int tile_h,
                                void* d_out_rgba, void* d_out_radiance, void* stream, rt_stats* stats) {
    int rc = check_render_args(ctx, cams, width, height, max_bounces, "rt_render_batch_rect_device");
    if (rc) return rc;
    if (n_frames < 1 || n_frames > kMaxBatch) {
        set_error("rt_render_batch_rect_device: n_frames must be in [1, %d], got %d", kMaxBatch, n_frames);
        return RT_ERR_INVALID_ARG;
    }
    if (x0 < 0 || y0 < 0 || tile_w < 0 || tile_h < 0 || x0 + tile_w > width || y0 + tile_h > height) {
        set_error("rt_render_batch_rect_device: rectangle (%d, %d) %d x %d outside the %d x %d frame", x0, y0, tile_w,
                  tile_h, width, height);
        return RT_ERR_INVALID_ARG;
    }
    if (tile_w == 0 || tile_h == 0) {
        if (stats) std::memset(stats, 0, sizeof *stats);
        return RT_OK;
    }
    PerDevice& p = ctx->dev[0];
    RT_HIP_CHECK(hipSetDevice(p.device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    // the rectangle's rows are one band of tile_h rows starting at y0
    rc = render_rows_on(ctx, p, cams, n_frames, width, height, max_bounces, tile_h, 1, 0, nullptr, tile_h,
                        static_cast<uchar4*>(d_out_rgba), static_cast<float*>(d_out_radiance), s, stats != nullptr, 0,
                        x0, y0, tile_w);
    if (rc) return rc;
    if (stats) {
        RT_HIP_CHECK(hipEventSynchronize(p.ev1));
        return collect_stats(ctx, p, (uint64_t)tile_w * tile_h * n_frames, stats, false);
    }
    return RT_OK;
}

int rt_render_batch_runs_device(rt_ctx* ctx, const rt_camera_ubo* cams, int n_frames, int width, int height,
                                int max_bounces, int band_h, const int32_t* band_lo, const int32_t* band_hi,
                                void* d_out_rgba, void* d_out_radiance, void* stream, rt_stats* stats) {
    int rc = check_render_args(ctx, cams, width, height, max_bounces, "rt_render_batch_runs_device");
    if (rc) return rc;
    if (n_frames < 1 || n_frames > kMaxBatch || !band_lo || !band_hi || band_h < 1 || height % band_h) {
        set_error("rt_render_batch_runs_device: need 1 <= n_frames <= %d, band_h dividing the height and both run "
                  "arrays", kMaxBatch);
        return RT_ERR_INVALID_ARG;
    }
    const int n_all = (height + band_h - 1) / band_h;
    int n_per = 0;
    for (int f = 0; f < n_frames; ++f) {
        if (band_lo[f] < 0 || band_hi[f] < band_lo[f] || band_hi[f] > n_all) {
            set_error("rt_render_batch_runs_device: frame %d's run [%d, %d) is not inside [0, %d)", f, band_lo[f],
                      band_hi[f], n_all);
            return RT_ERR_INVALID_ARG;
        }
        n_per = std::max(n_per, band_hi[f] - band_lo[f]);
    }
    if (n_per == 0) {
        if (stats) std::memset(stats, 0, sizeof *stats);
        return RT_OK;
    }
    // one band list per frame, -1 padded to the longest run, then each
    // frame's first output row (its rows follow the previous frame's)
    std::vector<int> list((size_t)n_frames * n_per + n_frames, -1);
    uint64_t pixels = 0;
    int row = 0;
    for (int f = 0; f < n_frames; ++f) {
        for (int b = band_lo[f]; b < band_hi[f]; ++b) list[(size_t)f * n_per + (b - band_lo[f])] = b;
        list[(size_t)n_frames * n_per + f] = row;
        const int rows_f = (band_hi[f] - band_lo[f]) * band_h;
        row += rows_f;
        pixels += (uint64_t)rows_f * (uint64_t)width;
    }
    PerDevice& p = ctx->dev[0];
    RT_HIP_CHECK(hipSetDevice(p.device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    rc = render_rows_on(ctx, p, cams, n_frames, width, height, max_bounces, band_h, 1, 0, &list, n_per * band_h,
                        static_cast<uchar4*>(d_out_rgba), static_cast<float*>(d_out_radiance), s, stats != nullptr,
                        n_per, 0, 0, 0, true);
    if (rc) return rc;
    if (stats) {
        RT_HIP_CHECK(hipEventSynchronize(p.ev1));
        return collect_stats(ctx, p, pixels, stats, false);
    }
    return RT_OK;
}

int rt_band_lists_rows(int height, int band_h, const int32_t* bands, int n_frames, int n_per) {
    if (height < 1 || band_h < 1 || height % band_h != 0 || n_frames < 1 || n_per < 1 || !bands) return -1;
    for (int f = 0; f < n_frames; ++f) {
        const int32_t* l = bands + (size_t)f * n_per;
        int k = 0;
        while (k < n_per && l[k] >= 0) ++k;                 // the list, then -1 padding only
        for (int j = k; j < n_per; ++j)
            if (l[j] != -1) return -1;
        if (rt_band_list_rows(height, band_h, l, k) < 0) return -1;
    }
    return n_per * band_h;                                  // every band is whole: the frame stride
}

int rt_render_batch_lists_device(rt_ctx* ctx, const rt_camera_ubo* cams, int n_frames, int width, int height,
                                 int max_bounces, int band_h, const int32_t* bands, int n_per,
                                 void* d_out_rgba, void* d_out_radiance, void* stream, rt_stats* stats) {
    int rc = check_render_args(ctx, cams, width, height, max_bounces, "rt_render_batch_lists_device");
    if (rc) return rc;
    if (n_frames < 1 || n_frames > kMaxBatch) {
        set_error("rt_render_batch_lists_device: n_frames must be in [1, %d], got %d", kMaxBatch, n_frames);
        return RT_ERR_INVALID_ARG;
    }
    const int rows = rt_band_lists_rows(height, band_h, bands, n_frames, n_per);
    if (rows < 0) {
        set_error("rt_render_batch_lists_device: bad band lists (height %d, band_h %d, %d per frame: band_h must "
                  "divide height; each frame's indices must increase and lie below height / band_h, then -1 "
                  "padding only)", height, band_h, n_per);
        return RT_ERR_INVALID_ARG;
    }
    uint64_t pixels = 0;
    for (int f = 0; f < n_frames; ++f) {
        const int32_t* l = bands + (size_t)f * n_per;
        int k = 0;
        while (k < n_per && l[k] >= 0) ++k;
        pixels += (uint64_t)rt_band_list_rows(height, band_h, l, k) * (uint64_t)width;
    }
    if (rows == 0) {
        if (stats) std::memset(stats, 0, sizeof *stats);
        return RT_OK;
    }
    PerDevice& p = ctx->dev[0];
    RT_HIP_CHECK(hipSetDevice(p.device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    const std::vector<int> list(bands, bands + (size_t)n_frames * n_per);
    rc = render_rows_on(ctx, p, cams, n_frames, width, height, max_bounces, band_h, 1, 0, &list, rows,
                        static_cast<uchar4*>(d_out_rgba), static_cast<float*>(d_out_radiance), s,
                        stats != nullptr, n_per);
    if (rc) return rc;
    if (stats) {
        RT_HIP_CHECK(hipEventSynchronize(p.ev1));
        return collect_stats(ctx, p, pixels, stats, false);
    }
    return RT_OK;
}

int rt_render(rt_ctx* ctx, const rt_camera_ubo* cam, int width, int height, int max_bounces,
              uint8_t* out_rgba, float* out_radiance, rt_stats* stats) {
    int rc = check_render_args(ctx, cam, width, height, max_bounces, "rt_render");
    if (rc) return rc;
    if (!out_rgba) { set_error("rt_render: out_rgba is required"); return RT_ERR_INVALID_ARG; }
    const int nd = (int)ctx->dev.size();
    // Device k renders the interleaved 16-row bands k, k+nd, ... (sky rows and
    // geometry rows spread evenly), into a packed buffer that is read back and
    // scattered to the bands' rows.
    const int bh = nd == 1 ? height : 16;
    std::vector<int> rows(nd);
    for (int k = 0; k < nd; ++k) rows[k] = rt_band_rows(height, bh, nd, k);
    for (int k = 0; k < nd; ++k) {
        if (rows[k] == 0) continue;
        PerDevice& p = ctx->dev[k];
        RT_HIP_CHECK(hipSetDevice(p.device));
        rc = ensure_out(p, (size_t)width * rows[k], out_radiance != nullptr);
        if (rc) return rc;
        rc = render_bands_on(ctx, p, cam, width, height, max_bounces, bh, nd, k, rows[k], p.d_rgba,
                             out_radiance ? p.d_rad : nullptr, p.stream, stats != nullptr);
        if (rc) return rc;
    }
    if (stats) std::memset(stats, 0, sizeof *stats);
    std::vector<uint8_t> stage_rgba;
    std::vector<float> stage_rad;
    for (int k = 0; k < nd; ++k) {
        if (rows[k] == 0) continue;
        PerDevice& p = ctx->dev[k];
        RT_HIP_CHECK(hipSetDevice(p.device));
        const size_t px = (size_t)width * rows[k];
        uint8_t* dst_rgba = out_rgba;
        float* dst_rad = out_radiance;
        if (nd > 1) {
            stage_rgba.resize(px * 4);
            dst_rgba = stage_rgba.data();
            if (out_radiance) { stage_rad.resize(px * 3); dst_rad = stage_rad.data(); }
        }
        RT_HIP_CHECK(hipMemcpyAsync(dst_rgba, p.d_rgba, px * 4, hipMemcpyDeviceToHost, p.stream));
        if (out_radiance)
            RT_HIP_CHECK(hipMemcpyAsync(dst_rad, p.d_rad, px * 12, hipMemcpyDeviceToHost, p.stream));
        RT_HIP_CHECK(hipStreamSynchronize(p.stream));
        if (nd > 1) {
            for (int ly = 0; ly < rows[k]; ++ly) {
                const int y = ((ly / bh) * nd + k) * bh + ly % bh;
                std::memcpy(out_rgba + (size_t)y * width * 4, dst_rgba + (size_t)ly * width * 4, (size_t)width * 4);
                if (out_radiance)
                    std::memcpy(out_radiance + (size_t)y * width * 3, dst_rad + (size_t)ly * width * 3,
                                (size_t)width * 12);
            }
        }
        if (stats) {
            rc = collect_stats(ctx, p, px, stats, true);
            if (rc) return rc;
        }
    }
    return RT_OK;
}

void* rt_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0 || hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess) {
        set_error("rt_host_alloc: could not pin %zu bytes", bytes);
        return nullptr;
    }
    return p;
}

void rt_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int rt_render_async(rt_ctx* ctx, const rt_camera_ubo* cam, int width, int height, int max_bounces,
                    uint8_t* out_rgba, uint64_t* ticket) {
    int rc = check_render_args(ctx, cam, width, height, max_bounces, "rt_render_async");
    if (rc) return rc;
    if (!out_rgba || !ticket) { set_error("rt_render_async: out_rgba and ticket are required"); return RT_ERR_INVALID_ARG; }
    const int nd = (int)ctx->dev.size();
    const int bh = nd == 1 ? height : 16;
    const int n_bands = (height + bh - 1) / bh;
    const size_t band_bytes = (size_t)bh * (size_t)width * 4;
    const uint64_t t = ctx->issued + 1;
    const int S = ctx->async_slots;
    const int slot = (int)(t % (uint64_t)S);
    for (int k = 0; k < nd; ++k) {
        const int rows = rt_band_rows(height, bh, nd, k);
        if (rows == 0) continue;
        PerDevice& p = ctx->dev[k];
        RT_HIP_CHECK(hipSetDevice(p.device));
        const size_t px = (size_t)width * rows;
        if (px > p.ring_cap) {                      // grow every slot once nothing is in flight
            for (int k2 = 0; k2 < kMaxSlots; ++k2)
                if (p.slot_stream[k2]) RT_HIP_CHECK(hipStreamSynchronize(p.slot_stream[k2]));
            RT_HIP_CHECK(hipStreamSynchronize(p.copy_stream));
            RT_HIP_CHECK(hipStreamSynchronize(p.copy_stream2));
            for (int k2 = 0; k2 < kMaxSlots; ++k2) {
                if (p.d_ring[k2]) (void)hipFree(p.d_ring[k2]);
                p.d_ring[k2] = nullptr;
            }
            p.ring_cap = px;
        }
        if (!p.d_ring[slot]) RT_HIP_CHECK(hipMalloc(&p.d_ring[slot], p.ring_cap * 4));
        // Each slot traces on its own stream (its own hardware queue with
        // GPU_MAX_HW_QUEUES >= slots + 2), so the frames in flight run at once.
        if (!p.slot_stream[slot]) RT_HIP_CHECK(hipStreamCreateWithFlags(&p.slot_stream[slot], hipStreamNonBlocking));
        const hipStream_t ts = p.slot_stream[slot];
        // The slot's previous frame must be read back before it is overwritten
        // (both halves, if it split its readback).
        RT_HIP_CHECK(hipStreamWaitEvent(ts, p.copied[slot], 0));
        if (p.slot_split[slot]) RT_HIP_CHECK(hipStreamWaitEvent(ts, p.copied2[slot], 0));
        // A frame that reads and writes per-device state shared by the slots
        // (the accumulation extension's running sums; the diagnostic records)
        // must not overlap the previous frame: its trace waits for that one.
        if (((ctx->ext & kExtAccumulate) || ctx->diag) && t > 1) {
            const int prev = (int)((t - 1) % (uint64_t)S);
            if (p.slot_ticket[prev] == t - 1) RT_HIP_CHECK(hipStreamWaitEvent(ts, p.traced[prev], 0));
        }
        ctx->in_async = S;
        rc = render_bands_on(ctx, p, cam, width, height, max_bounces, bh, nd, k, rows, p.d_ring[slot], nullptr, ts,
                             false);
        ctx->in_async = 0;
        if (rc) return rc;
        RT_HIP_CHECK(hipEventRecord(p.traced[slot], ts));
        // Copies run in ticket order on the one copy stream, whatever order the
        // traces finish in.  copy_stream2 (a split readback's second half) is
        // touched only by the frames that split: a join on an idle stream per
        // frame costs the pipelined loop time for nothing.
        RT_HIP_CHECK(hipStreamWaitEvent(p.copy_stream, p.traced[slot], 0));
        const bool split = nd == 1 && ctx->copy_streams == 2 && rows > 1;
        if (split) RT_HIP_CHECK(hipStreamWaitEvent(p.copy_stream2, p.traced[slot], 0));
        if (split) {
            // the frame's top and bottom halves on two copy streams, so two copy
            // engines read the frame back at once
            const size_t top = (size_t)width * (size_t)(rows / 2) * 4;
            RT_HIP_CHECK(hipMemcpyAsync(out_rgba, p.d_ring[slot], top, hipMemcpyDeviceToHost, p.copy_stream));
            RT_HIP_CHECK(hipMemcpyAsync(out_rgba + top, reinterpret_cast<uint8_t*>(p.d_ring[slot]) + top,
                                        px * 4 - top, hipMemcpyDeviceToHost, p.copy_stream2));
        } else if (nd == 1) {
            RT_HIP_CHECK(hipMemcpyAsync(out_rgba, p.d_ring[slot], px * 4, hipMemcpyDeviceToHost, p.copy_stream));
        } else {
            // bands k, k+nd, ...: every full band in one strided copy, a partial last band on its own
            const int n_k = (n_bands - k + nd - 1) / nd;
            const int last = k + (n_k - 1) * nd;
            const bool partial = (last + 1) * bh > height;
            const int full = partial ? n_k - 1 : n_k;
            if (full > 0)
                RT_HIP_CHECK(hipMemcpy2DAsync(out_rgba + (size_t)k * band_bytes, (size_t)nd * band_bytes,
                                              p.d_ring[slot], band_bytes, band_bytes, (size_t)full,
                                              hipMemcpyDeviceToHost, p.copy_stream));
            if (partial)
                RT_HIP_CHECK(hipMemcpyAsync(out_rgba + (size_t)last * band_bytes,
                                            reinterpret_cast<uint8_t*>(p.d_ring[slot]) + (size_t)full * band_bytes,
                                            (size_t)(height - last * bh) * width * 4, hipMemcpyDeviceToHost,
                                            p.copy_stream));
        }
        RT_HIP_CHECK(hipEventRecord(p.copied[slot], p.copy_stream));
        if (split) {
            RT_HIP_CHECK(hipEventRecord(p.copied2[slot], p.copy_stream2));
            p.last_split_t = t;
            p.last_split_slot = slot;
        }
        p.slot_split[slot] = split;
        p.slot_ticket[slot] = t;
    }
    ctx->issued = t;
    *ticket = t;
    return RT_OK;
}

// The events that cover frame `ticket` on device p.  Copies complete in
// ticket order on copy_stream, so the copy event of the slot with the smallest
// ticket >= this one covers it (e1; null: the device has no rows of that
// frame, and copy_stream itself is waited on).  A split frame's second half
// runs in ticket order on copy_stream2, so the copied2 event of the slot with
// the smallest SPLIT ticket >= this one covers it (e2; the requested frame's
// own when its slot still holds it), not the newest split frame's, which
// would wait for every later frame in flight.  If no slot holds a split frame
// >= ticket any more but one was issued, the newest split event (kept until
// it is re-recorded) covers it.
static void cover_events(const PerDevice& p, uint64_t ticket, hipEvent_t* e1, hipEvent_t* e2) {
    int best = -1, best2 = -1;
    for (int k2 = 0; k2 < kMaxSlots; ++k2) {
        if (p.slot_ticket[k2] < ticket) continue;
        if (best < 0 || p.slot_ticket[k2] < p.slot_ticket[best]) best = k2;
        if (p.slot_split[k2] && (best2 < 0 || p.slot_ticket[k2] < p.slot_ticket[best2])) best2 = k2;
    }
    *e1 = best >= 0 ? p.copied[best] : nullptr;
    *e2 = best2 >= 0 ? p.copied2[best2]
                     : (p.last_split_t >= ticket && p.last_split_slot >= 0 ? p.copied2[p.last_split_slot] : nullptr);
}

static int check_ticket(const rt_ctx* ctx, uint64_t ticket, const char* fn) {
    if (ticket == 0 || ticket > ctx->issued) {
        set_error("%s: ticket %llu was not issued (last %llu)", fn, (unsigned long long)ticket,
                  (unsigned long long)ctx->issued);
        return RT_ERR_INVALID_ARG;
    }
    return RT_OK;
}

int rt_render_wait(rt_ctx* ctx, uint64_t ticket) {
    if (!ctx) { set_error("rt_render_wait: null context"); return RT_ERR_INVALID_ARG; }
    if (int rc = check_ticket(ctx, ticket, "rt_render_wait")) return rc;
    for (PerDevice& p : ctx->dev) {
        RT_HIP_CHECK(hipSetDevice(p.device));
        hipEvent_t e1, e2;
        cover_events(p, ticket, &e1, &e2);
        if (e1) RT_HIP_CHECK(hipEventSynchronize(e1));
        else RT_HIP_CHECK(hipStreamSynchronize(p.copy_stream));
        if (e2) RT_HIP_CHECK(hipEventSynchronize(e2));
    }
    return RT_OK;
}

int rt_render_poll(rt_ctx* ctx, uint64_t ticket, int* done) {
    if (!ctx || !done) { set_error("rt_render_poll: null argument"); return RT_ERR_INVALID_ARG; }
    if (int rc = check_ticket(ctx, ticket, "rt_render_poll")) return rc;
    *done = 0;
    for (PerDevice& p : ctx->dev) {
        RT_HIP_CHECK(hipSetDevice(p.device));
        hipEvent_t e1, e2;
        cover_events(p, ticket, &e1, &e2);
        for (int k = 0; k < 2; ++k) {
            const hipError_t q = k == 0 ? (e1 ? hipEventQuery(e1) : hipStreamQuery(p.copy_stream))
                                        : (e2 ? hipEventQuery(e2) : hipSuccess);
            if (q == hipErrorNotReady) return RT_OK;
            RT_HIP_CHECK(q);
        }
    }
    *done = 1;
    return RT_OK;
}

int rt_set_option(rt_ctx* ctx, const char* name, int64_t value) {
    if (!ctx || !name) { set_error("rt_set_option: null argument"); return RT_ERR_INVALID_ARG; }
    static const char* const archived[] = {"shade_min", "blocks_per_cu", "seg_limit", "heavy_budget", "prio_after"};
    for (const char* a : archived)
        if (std::strcmp(name, a) == 0) {
            set_error("rt_set_option: %s belonged to a schedule archived in round 3 (profiles/r03/archive)", name);
            return RT_ERR_INVALID_ARG;
        }
    if (std::strcmp(name, "kernel") == 0 && value == 0) {
        // the one kernel (kernels 1-3, persistent / split / tiered, are archived)
    } else if (std::strcmp(name, "coop_lanes") == 0 && value >= -1 && value <= 64) {
        ctx->coop_lanes = (int)value;
    } else if (std::strcmp(name, "extensions") == 0 && value >= 0 && value <= 15) {
        ctx->ext = (int)value;
    } else if (std::strcmp(name, "walk") == 0 && (value == 0 || value == 2)) {
        ctx->walk = (int)value;
    } else if (std::strcmp(name, "coop_window") == 0 && (value == 0 || value == 32 || value == 64)) {
        ctx->coop_window = (int)value;
    } else if (std::strcmp(name, "coop_walk") == 0 && (value == 0 || value == 1)) {
        ctx->coop_walk = (int)value;
    } else if (std::strcmp(name, "block_waves") == 0 && (value == 1 || value == 4)) {
        ctx->block_waves = (int)value;
    } else if (std::strcmp(name, "heavy_first") == 0 && (value == 0 || value == 1)) {
        ctx->heavy_first = (int)value;
    } else if (std::strcmp(name, "heavy_tiles") == 0 && value >= -1 && value <= (1 << 20)) {
        ctx->heavy_tiles = (int)value;
    } else if (std::strcmp(name, "heavy_factor") == 0 && value >= 10 && value <= 100000) {
        ctx->heavy_factor = (int)value;
    } else if (std::strcmp(name, "heavy_pixels") == 0 && (value == 0 || value == 1)) {
        ctx->heavy_pixels = (int)value;
    } else if (std::strcmp(name, "heavy_pixel_factor") == 0 && value >= 1 && value <= 100000) {
        ctx->heavy_pixel_factor = (int)value;
    } else if (std::strcmp(name, "reuse_order") == 0 && (value == 0 || value == 1)) {
        ctx->reuse_order = (int)value;
    } else if (std::strcmp(name, "heavy_cap") == 0 && value >= 1 && value <= 100) {
        ctx->heavy_cap = (int)value;
    } else if (std::strcmp(name, "async_slots") == 0 && value >= 1 && value <= kMaxSlots) {
        ctx->async_slots = (int)value;
    } else if (std::strcmp(name, "copy_streams") == 0 && (value == 1 || value == 2)) {
        ctx->copy_streams = (int)value;
    } else if (std::strcmp(name, "concurrent_launches") == 0 && value >= 1 && value <= 64) {
        ctx->concurrent_launches = (int)value;
    } else if (std::strcmp(name, "learn_cost") == 0 && (value == 0 || value == 1)) {
        ctx->learn_cost = (int)value;
    } else if (std::strcmp(name, "order_frames") == 0 && (value == 0 || value == 1)) {
        ctx->order_frames = (int)value;
    } else if (std::strcmp(name, "order_split") == 0 && value >= 0 && value <= 100) {
        ctx->order_split = (int)value;
    } else if (std::strcmp(name, "learn_alone") == 0 && (value == 0 || value == 1)) {
        ctx->learn_alone = (int)value;
    } else if (std::strcmp(name, "xcd_order") == 0 && value >= 0 && value <= 4096) {
        ctx->xcd_order = (int)value;
    } else if (std::strcmp(name, "accel_octants") == 0 && value >= 0 && value <= 7) {
        ctx->accel_octants = (int)value;
    } else if (std::strcmp(name, "learn_device") == 0 && (value == 0 || value == 1)) {
        ctx->learn_device = (int)value;
    } else if (std::strcmp(name, "leaf_align") == 0 && value >= 0 && value <= 2) {
        ctx->leaf_align = (int)value;                   // takes effect at the next rt_upload_scene
    } else if (std::strcmp(name, "accel") == 0 && (value == 0 || value == 1 || value == 8)) {
        ctx->accel = (int)value;                        // takes effect at the next rt_upload_scene
    } else if (std::strcmp(name, "split_bounce") == 0 && value >= 0 && value <= 64) {
        ctx->split_bounce = (int)value;
    } else if (std::strcmp(name, "accel_half") == 0 && (value == 0 || value == 1)) {
        ctx->accel_half = (int)value;                   // takes effect at the next rt_upload_scene
    } else if (std::strcmp(name, "accel_wide") == 0 && (value == 0 || value == 1)) {
        ctx->accel_wide = (int)value;                   // takes effect at the next rt_upload_scene
    } else if (std::strcmp(name, "heavy_stream") == 0 && value >= 0 && value <= 2) {
        ctx->heavy_stream = (int)value;
    } else if (std::strcmp(name, "graph") == 0 && (value == 0 || value == 1)) {
        ctx->graph = (int)value;
    } else if (std::strcmp(name, "diag") == 0 && (value == 0 || value == 1)) {
        ctx->diag = (int)value;
    } else if (std::strcmp(name, "wave_tile") == 0 && value >= -1 && value <= 3) {
        ctx->wave_tile = (int)value;
    } else {
        set_error("rt_set_option: unknown option or bad value: %s = %lld", name, (long long)value);
        return RT_ERR_INVALID_ARG;
    }
    return RT_OK;
}

int rt_get_option(rt_ctx* ctx, const char* name, int64_t* value) {
    if (!ctx || !name || !value) { set_error("rt_get_option: null argument"); return RT_ERR_INVALID_ARG; }
    if (std::strcmp(name, "kernel") == 0) *value = 0;
    else if (std::strcmp(name, "wave_tile") == 0) *value = ctx->wave_tile;
    else if (std::strcmp(name, "wave_tile_used") == 0)
        *value = ctx->dev.empty() ? 0 : wave_tile_of(ctx, ctx->dev[0]);
    else if (std::strcmp(name, "coop_lanes") == 0) *value = ctx->coop_lanes;
    else if (std::strcmp(name, "walk") == 0) *value = ctx->walk;
    else if (std::strcmp(name, "coop_walk") == 0) *value = ctx->coop_walk;
    else if (std::strcmp(name, "coop_window") == 0) *value = ctx->coop_window;
    else if (std::strcmp(name, "coop_window_used") == 0)
        *value = ctx->dev.empty() ? 0 : coop_window_of(ctx, ctx->dev[0]);
    else if (std::strcmp(name, "block_waves") == 0) *value = ctx->block_waves;
    else if (std::strcmp(name, "heavy_first") == 0) *value = ctx->heavy_first;
    else if (std::strcmp(name, "heavy_tiles") == 0) *value = ctx->heavy_tiles;
    else if (std::strcmp(name, "heavy_stream") == 0) *value = ctx->heavy_stream;
    else if (std::strcmp(name, "graph") == 0) *value = ctx->graph;
    else if (std::strcmp(name, "learn_cost") == 0) *value = ctx->learn_cost;
    else if (std::strcmp(name, "order_split") == 0) *value = ctx->order_split;
    else if (std::strcmp(name, "learn_alone") == 0) *value = ctx->learn_alone;
    else if (std::strcmp(name, "xcd_order") == 0) *value = ctx->xcd_order;
    else if (std::strcmp(name, "accel_octants") == 0) *value = ctx->accel_octants;
    else if (std::strcmp(name, "learn_device") == 0) *value = ctx->learn_device;
    else if (std::strcmp(name, "leaf_align") == 0) *value = ctx->leaf_align;
    else if (std::strcmp(name, "accel") == 0) *value = ctx->accel;
    else if (std::strcmp(name, "accel_half") == 0) *value = ctx->accel_half;
    else if (std::strcmp(name, "split_bounce") == 0) *value = ctx->split_bounce;
    else if (std::strcmp(name, "accel_half_used") == 0) *value = ctx->dev.empty() ? 0 : ctx->dev[0].scene.half;
    else if (std::strcmp(name, "accel_wide") == 0) *value = ctx->accel_wide;
    else if (std::strcmp(name, "accel_wide_used") == 0) *value = ctx->dev.empty() ? 0 : ctx->dev[0].scene.wide;
    else if (std::strcmp(name, "walk_bytes") == 0) *value = ctx->dev.empty() ? 0 : (int64_t)walk_bytes(ctx->dev[0]);
    else if (std::strcmp(name, "accel_used") == 0) *value = ctx->dev.empty() ? 0 : ctx->dev[0].scene.n_layouts;
    else if (std::strcmp(name, "leaf_align_used") == 0) *value = ctx->dev.empty() ? 0 : ctx->dev[0].scene.padded;
    else if (std::strcmp(name, "heavy_factor") == 0) *value = ctx->heavy_factor;
    else if (std::strcmp(name, "concurrent_launches") == 0) *value = ctx->concurrent_launches;
    else if (std::strcmp(name, "async_slots") == 0) *value = ctx->async_slots;
    else if (std::strcmp(name, "copy_streams") == 0) *value = ctx->copy_streams;
    else if (std::strcmp(name, "heavy_cap") == 0) *value = ctx->heavy_cap;
    else if (std::strcmp(name, "reuse_order") == 0) *value = ctx->reuse_order;
    else if (std::strcmp(name, "heavy_pixels") == 0) *value = ctx->heavy_pixels;
    else if (std::strcmp(name, "heavy_pixel_factor") == 0) *value = ctx->heavy_pixel_factor;
    else if (std::strcmp(name, "heavy_pixels_used") == 0) *value = ctx->dev.empty() ? 0 : ctx->dev[0].last_heavy_px;
    else if (std::strcmp(name, "heavy_tiles_used") == 0) *value = ctx->dev.empty() ? 0 : ctx->dev[0].last_heavy;
    else if (std::strcmp(name, "plain_kernels") == 0) *value = ctx->dev.empty() ? 0 : (int64_t)ctx->dev[0].plain_kernels;
    else if (std::strcmp(name, "extensions") == 0) *value = ctx->ext;
    else if (std::strcmp(name, "hw_queues") == 0) *value = ctx->hw_queues;
    else if (std::strcmp(name, "order_frames") == 0) *value = ctx->order_frames;
    // 1 when rt_render_async's slots cannot each have a hardware queue of their
    // own (async_slots + 2 > hw_queues: the slots' traces then share queues and
    // run one after another); start the host with GPU_MAX_HW_QUEUES >= slots + 2
    else if (std::strcmp(name, "queues_short") == 0) *value = ctx->async_slots + 2 > ctx->hw_queues ? 1 : 0;
    else { set_error("rt_get_option: unknown option %s", name); return RT_ERR_INVALID_ARG; }
    return RT_OK;
}

int rt_diag_copy(rt_ctx* ctx, void* dst, size_t cap_words, size_t* n_words) {
    if (!ctx || !n_words) { set_error("rt_diag_copy: null argument"); return RT_ERR_INVALID_ARG; }
    PerDevice& p = ctx->dev[0];
    *n_words = p.diag_used;
    if (dst && p.d_diag && p.diag_used) {
        RT_HIP_CHECK(hipSetDevice(p.device));
        RT_HIP_CHECK(hipDeviceSynchronize());
        RT_HIP_CHECK(hipMemcpy(dst, p.d_diag, std::min(cap_words, p.diag_used) * 8, hipMemcpyDeviceToHost));
    }
    return RT_OK;
}

static int wire_args(const void* a, const void* b, size_t n_px, const char* fn) {
    if (n_px && (!a || !b)) {
        set_error("%s: null buffer", fn);
        return RT_ERR_INVALID_ARG;
    }
    return RT_OK;
}

int rt_pack_rgb(const void* d_rgba, void* d_rgb, size_t n_px, void* stream) {
    if (int rc = wire_args(d_rgba, d_rgb, n_px, "rt_pack_rgb")) return rc;
    if ((uintptr_t)d_rgba % 16 || (uintptr_t)d_rgb % 4) {
        set_error("rt_pack_rgb: the RGBA8 buffer must be 16-B aligned and the RGB buffer 4-B aligned");
        return RT_ERR_INVALID_ARG;
    }
    if (n_px) RT_HIP_CHECK(wire_pack(d_rgba, d_rgb, n_px, static_cast<hipStream_t>(stream)));
    return RT_OK;
}

int rt_unpack_rgb(const void* d_rgb, void* d_rgba, size_t n_px, void* stream) {
    if (int rc = wire_args(d_rgb, d_rgba, n_px, "rt_unpack_rgb")) return rc;
    if ((uintptr_t)d_rgba % 16 || (uintptr_t)d_rgb % 4) {
        set_error("rt_unpack_rgb: the RGBA8 buffer must be 16-B aligned and the RGB buffer 4-B aligned");
        return RT_ERR_INVALID_ARG;
    }
    if (n_px) RT_HIP_CHECK(wire_unpack(d_rgb, d_rgba, n_px, static_cast<hipStream_t>(stream)));
    return RT_OK;
}

int rt_accel_records(const void* vertices, size_t vertex_bytes, const void* materials, size_t material_bytes,
                     const void* bvh_nodes, size_t bvh_bytes, int n_layouts, uint32_t* out_words, size_t cap_words,
                     size_t* n_words, int32_t info[8]) {
    HostScene hs;
    const char* err = nullptr;
    int rc = build_host_scene(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, bvh_bytes, &hs, &err);
    if (rc != RT_OK) { set_error("rt_accel_records: %s", err); return rc; }
    const size_t reach = (size_t)hs.end * RT_NODE_RECORD_BYTES;    // the root's subtree only
    free_host_scene(&hs);
    AccelHost ah;
    std::string msg;
    const int nl = n_layouts & ~(RT_ACCEL_FORMAT_HALF | RT_ACCEL_FORMAT_WIDE);
    if ((nl != 1 && nl != 8) || ((n_layouts & RT_ACCEL_FORMAT_HALF) && (n_layouts & RT_ACCEL_FORMAT_WIDE))) {
        set_error("rt_accel_records: n_layouts must be 1 or 8, with at most one format flag");
        return RT_ERR_INVALID_ARG;
    }
    rc = accel_build_fit(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, reach, nl, &ah, &msg,
                         (n_layouts & RT_ACCEL_FORMAT_HALF) ? 1 : (n_layouts & RT_ACCEL_FORMAT_WIDE) ? 2 : 0,
                         accel_cap_slots());
    if (rc == kAccelTooBig) {                      // rt_upload_scene walks the reference's tree: no records
        if (n_words) *n_words = 0;
        if (info) {
            for (int k = 0; k < 8; ++k) info[k] = 0;
        }
        return RT_OK;
    }
    if (rc != 0) {
        set_error("rt_accel_records: %s", msg.c_str());
        return RT_ERR_BAD_SCENE;
    }
    if (n_words) *n_words = ah.rec.size();
    if (info) {
        info[0] = ah.n_layouts; info[1] = ah.slots; info[2] = ah.root_leaf;
        info[3] = ah.n_prims; info[4] = ah.n_inputs; info[5] = ah.depth;
        info[6] = ah.max_class; info[7] = ah.n_thin;
    }
    if (out_words) std::memcpy(out_words, ah.rec.data(), std::min(cap_words, ah.rec.size()) * sizeof(uint32_t));
    return RT_OK;
}

int rt_scene_validate(const void* vertices, size_t vertex_bytes, const void* materials, size_t material_bytes,
                      const void* bvh_nodes, size_t bvh_bytes, size_t* n_nodes, int* max_depth) {
    HostScene hs;
    const char* err = nullptr;
    int rc = build_host_scene(vertices, vertex_bytes, materials, material_bytes, bvh_nodes, bvh_bytes, &hs, &err);
    if (rc != RT_OK) { set_error("rt_scene_validate: %s", err); return rc; }
    if (n_nodes) *n_nodes = (size_t)hs.end;
    if (max_depth) *max_depth = hs.max_depth;
    free_host_scene(&hs);
    return RT_OK;
}

}  // extern "C"
