// rt_internal.h — shared declarations of the gfx950 path-trace backend.
//
// Device layout of a scene (built once per rt_upload_scene from the
// reference's 48-B node / 48-B vertex / 16-B material records):
//
//   nodes : 2 x float4 per node (32 B), in the reference's preorder
//           [0] = (bbox_min.xyz, skip | L(skip) << 31)
//           [1] = (bbox_max.xyz, L(i+1) | L(i) << 1)
//           skip = first node after this subtree; L(j) = "node j is a leaf".
//           The left child of an internal node i is i+1 (BVHFlattener.java:51-75:
//           myIndex = currentNodeIndex++ and the left subtree is flattened
//           first), so the reference's stack DFS (compute_dynamic_ray.comp:185-210:
//           push right, push left) visits nodes in preorder, skipping the
//           subtree of every node whose box test fails.  "next = hit ? i+1 :
//           skip" replays exactly that visit sequence with no stack at all, and
//           the L bits tell a walker whether the node it moves to is a leaf, so
//           it fetches that leaf's triangle together with the node (one memory
//           round trip per visit).
//   leafs : 3 x float4 per NODE index (48 B; meaningful at leaves only)
//           [0] = (v0.xyz, triangle index) [1] = (e1.xyz, 0) [2] = (e2.xyz, 0)
//           e1 = v1-v0, e2 = v2-v0 are the values hit_triangle computes
//           (compute_dynamic_ray.comp:106-107), evaluated once on the host in
//           IEEE binary32: the same bits.
//   pairs : 4 x float4 per NODE index (64 B; meaningful at internal nodes only):
//           the boxes of both children of node i and where they are
//           [0] = (L.min.xyz, R.min.x) [1] = (L.max.xyz, R.min.y)
//           [2] = (R.max.xyz, R.min.z) [3] = (R | L(R) << 31, L(i+1), skip(i), 0)
//           with L = i+1 and R = the right child.  The frontier walk (heavy
//           pixels, option coop_walk 1) expands a hit internal node by
//           loading this one record and testing both children's boxes.
//   norms : 1 x float4 per flattened triangle: normalize(cross(e1,e2)) (:124),
//           likewise precomputed; read once per hit when shading.
//   mats  : 1 x float4 per flattened triangle (albedo.rgb, type)
#pragma once
#include <cstdint>
#include <cstddef>
#include <hip/hip_runtime.h>

#include "../../include/rtamd.h"

namespace rtamd {

constexpr int kShadeStride = 2;

struct DevScene {
    int      n_nodes = 0;     // nodes in the compact array
    int      end     = 0;     // traversal ends when the node index reaches this (= skip of root)
    int      n_tris  = 0;
    int      root_leaf = 0;   // L(0)
    float    root_box[6] = {0, 0, 0, 0, 0, 0};   // node 0's min.xyz, max.xyz (kernel argument)
    float4*  nodes   = nullptr;
    float4*  leafs   = nullptr;
    float4*  pairs   = nullptr;
    // walk 2's records (the lockstep walk and the cooperative tail), 32-B
    // slots: the reference's preorder with every leaf's triangle inlined after
    // its box.  An internal node takes one slot, (min.xyz, skip slot |
    // L(skip) << 31), (max.xyz, L(i+1) | L(i) << 1); a leaf two, (min.xyz,
    // triangle index | 1 << 30 | L(i+1) << 31), (max.xyz, v0.x), then
    // (v0.yz, e1.xy), (e1.z, e2.xyz).  slot(i) = i + the leaves before i, so
    // an internal node's left child (i+1) is the next slot and a leaf's
    // successor (its skip, i+1) the slot after its two: only the internal
    // skip is stored.  A leaf visit reads its node and triangle from one
    // 64-B run (they were two arrays), sibling leaves sit side by side, and
    // the records take 32 B per node + 32 B per leaf instead of 64 B per node
    // (config 5: 100 MB instead of 134 MB).  Bit 30 of word [0].w is L(i) for
    // every node.  end2 = the slots; slot_node = the node index of a node's
    // first slot (the frontier tail's hand-off), -1 on a leaf's second slot.
    float4*  walk    = nullptr;
    int*     slot_node = nullptr;
    int*     node_slot = nullptr;   // slot(i) of node i (walk 0 hands its node index to the windows tail)
    int      end2    = 0;
    int      padded  = 0;   // 1: the walk records hold pad slots (leaf_align)
    // Option accel (accel_build.h): walk = the accel records,
    // n_layouts (1 or 8) layouts of layout_slots slots each (end2 = their
    // total, end = layout_slots), and the reference's walk records beside
    // them for the fallback (a segment whose hit lies before its own box's
    // t_enter is walked again in the reference's order): walk_ref, end2_ref
    // slots (pad slots as `ref_padded`).  n_layouts 0: no accel.
    int      n_layouts = 0;
    int      layout_slots = 0;
    int      wide = 0;          // accel format 2: the 4-wide tree, 64-B records (end2 = records)
    int      half = 0;          // accel format 1: 16-B slots, half-precision internal boxes (accel_build.h);
                                //   layout_slots and end2 then count 16-B slots
    float    relax_half = 0.0f;  // format 1: every internal node's margin factor (AccelHost::relax_max)
    int      root_enter = 0;     // format 0: the walk starts inside the root (its slab test skipped)
    int      root_first_leaf = 0;   // bit o: layout o's root's first child is a leaf
    int      oct_mask = 7;       // 8 layouts: a ray walks layout (its octant & oct_mask) (option accel_octants)
    float4*  walk_ref = nullptr;
    int      end2_ref = 0;
    int      ref_padded = 0;
    // norms and mats interleave in one allocation (kShadeStride float4 per
    // triangle: normal, then albedo/type), so shading a hit touches one 32-B
    // record; norms points at the allocation, mats one float4 in
    float4*  norms   = nullptr;
    float4*  mats    = nullptr;
    // extension kExtSpheres: 2 x float4 per sphere (centre.xyz, radius),
    // (albedo.rgb, type); n_spheres is 0 unless the extension is on
    const float4* spheres = nullptr;
    int      n_spheres = 0;
};

struct Counters {               // device-side work counters (see rt_stats)
    unsigned long long segments;
    unsigned long long node_visits;
    unsigned long long tri_tests;
    unsigned long long mat_reads;
};

struct CamF {                   // the four vec3 of the CameraUBO
    float ox, oy, oz;
    float lx, ly, lz;
    float hx, hy, hz;
    float vx, vy, vz;
};

// Non-reference extensions (option "extensions", off by
// default, kernel 0 only).  The reference has none of them (SURVEY.md §0 facts
// 3-4); oracle/rt_oracle.h ORC_EXT_* states the same semantics.
constexpr int kExtSkyToggle = 1;    // a miss is black when sky_enabled == 0
constexpr int kExtEmissive = 2;     // a type-3 hit ends the path with attenuation * albedo
constexpr int kExtAccumulate = 4;   // seed += frame_count*W*H; output sqrt(mean of linear colour)
constexpr int kExtSpheres = 8;      // spheres (rt_upload_spheres) after the BVH walk, in index order

constexpr int kMaxBatch = 16;  // frames per launch (rt_render_batch_device)

struct TraceArgs {
    DevScene scene;
    CamF     cams[kMaxBatch];   // frame f of the batch is seen through cams[f]
    int      n_frames;          // frames in the launch (1..kMaxBatch): the same rows of each
    int      tiles_y;           // wave-tile rows per frame (launcher-internal: ceil(th / tile height))
    int      width, height;     // full frame
    int      max_bounces;
    int      x0, y0, tw, th;    // columns [x0, x0+tw); th local rows per frame
    // Local row ly is frame row y0 + ((ly / band_h) * band_stride + band_off) * band_h + ly % band_h:
    // a plain tile is band_h = th, band_stride = 1, band_off = 0; rank r of N
    // interleaved 16-row bands is band_h = 16, band_stride = N, band_off = r.
    // With band_list (device, nullable) it is band_list[ly / band_h] * band_h + ly % band_h; with
    // list_stride > 0 frame f reads its own list at band_list + f * list_stride, whose -1 entries
    // (trailing padding) and rows past the frame are not traced.
    int      band_h, band_stride, band_off;
    const int* band_list;
    // Outputs: n_frames x th x tw pixels, frame f's local row ly at row f * th + ly
    uchar4*  out_rgba;          // nullable
    float*   out_rad;           // 3 floats per pixel, nullable
    Counters* counters;         // nullable
    int      wave_tile;         // wave tile (8<<s) x (8>>s), s in 0..3
    unsigned long long* diag;   // diagnostics: 8 words per wave, or null
    int      coop_lanes;        // finish a wave's walks cooperatively once at most
                                //   this many lanes are still walking (0 = never)
    int      ext;               // non-reference extensions, kExt* bits (0 = the reference)
    int      sky_enabled;       // CameraUBO.sky_enabled (@68), read only with kExtSkyToggle
    int      frame_count;       // CameraUBO.frame_count (@64), read only with kExtAccumulate
    float*   accum;             // kExtAccumulate: running linear-colour sums, 3 floats per pixel (tw*th)
    int      walk;              // 0 = one node per step (nodes/leafs), 2 = the same software-pipelined
                                //   over the compact records (nodes2/leafs2; default)
    int      block_waves;       // waves per workgroup, 4 (256 threads) or 1 (64 threads)
    const int* tile_order;      // block_waves 1: workgroup k traces wave tile tile_order[k] (or k)
    int      tiles_x;           // with tile_order (1-D grid): wave tiles per tile row
    int      split_n;           // with tile_order: the first split_n tiles of the order are traced
                                //   one pixel per wave (64 workgroups each; launcher-internal)
    int      heavy_tiles;       // with tile_order: the first heavy_tiles tiles run in that split
                                //   mode as a concurrent launch on aux_stream (fork ev_fork, join ev_join)
    int      heavy_fused;       // with heavy_tiles: 1 = the heavy tiles' one-pixel workgroups come
                                //   first in the same launch (option heavy_stream 2), no aux stream
    const int* heavy_px;        // fused, with tile_order: heavy pixels (tile * 64 + lane), traced one
    int      n_heavy_px;        //   per wave by the first n_heavy_px workgroups of the launch
    const unsigned long long* tile_mask;   // per tile: the lanes (heavy pixels) its tile wave skips, or null
    unsigned* diag_lane;        // learning launch: each pixel's walk length (64 per wave), or null
    hipStream_t aux_stream;
    hipEvent_t ev_fork, ev_join;
    int      coop_walk;         // cooperative tail: 0 = 64-node preorder windows (coop_walk),
                                //   1 = preorder frontier (frontier_walk)
    int      coop_win = 64;     // coop_walk's window: 64 or 32 slots (option coop_window)
    int      list_stride;       // band_list per frame: frame f's at band_list + f * list_stride
    const int* row_off = nullptr;   // per frame: its first output row (null: f * th); device memory
                                //   (0 = one list for every frame of the launch)
    // Split launch (option split_bounce, accel walk): kernel 1
    // packs each wave's paths still alive at bounce split_bounce into the
    // wave's 64 ray slots (3 float4 each) and writes the wave's count; a scan
    // makes q_prefix (q_waves + 1 entries); kernel 2 finishes the paths 64 per
    // wave in slot order.  q_slots null: one kernel.
    int      split_bounce = 0;
    float4*  q_slots = nullptr;
    unsigned* q_count = nullptr;
    unsigned* q_prefix = nullptr;
    int      q_waves = 0;       // the slots' capacity in waves (launch_trace: kernel 1's waves)
    int      q_grid = 0;        // kernel 2's one-wave workgroups
    void*    q_temp = nullptr;  // the scan's temporary storage (rocPRIM), q_temp_bytes
    size_t   q_temp_bytes = 0;
};

// Host-side compact-scene build from the reference records; validates the
// buffers.  Returns RT_OK or RT_ERR_BAD_SCENE with a message in *err.
struct HostScene {
    int n_nodes = 0, end = 0, n_tris = 0, max_depth = 0, root_leaf = 0;
    float root_box[6] = {0, 0, 0, 0, 0, 0};
    float4* nodes = nullptr;    // 2*n_nodes
    float4* leafs = nullptr;    // 3*n_nodes
    float4* pairs = nullptr;    // 4*n_nodes
    float4* norms = nullptr;    // n_tris
    float4* mats  = nullptr;    // n_tris
};
int build_host_scene(const void* vertices, size_t vertex_bytes,
                     const void* materials, size_t material_bytes,
                     const void* bvh_nodes, size_t bvh_bytes,
                     HostScene* out, const char** err);
void free_host_scene(HostScene* s);

// A learning launch's walk length of a pixel traced by a one-pixel heavy wave
// (its lockstep length is unknown there): above any real length, so it stays
// among the heavy pixels (rt_learn.hip).
constexpr unsigned kLearnHeavyMark = 0x3FFFFFFFu;

// Device-side heavy-first learning (rt_learn.hip): the order, heavy pixels and
// tile masks from a learning launch's diagnostic records, computed on the
// stream that ran it, with no host synchronisation.
struct LearnParams {
    int      n;              // tiles of the launch (records at rec_off + t, pixels at t * 64 + lane)
    int      rec_off;        // heavy-pixel waves ahead of the tile records (a fused launch in an order)
    int      learn_cost;     // 0 = lockstep steps + 2 x windows, 1 = wave duration
    int      order_split;    // percent (0 = every tile by cost)
    double   bar_scale;      // heavy-pixel bar = bar_scale x total steps
    int      cap;            // at most this many heavy pixels
    // option xcd_order (> 0, n a multiple of 8): tile_order position k runs on
    // XCD k % 8 (workgroups are dealt round-robin); XCD c gets the c-th eighth
    // of the tiles in the order of (row class, row, frame, column), a row's
    // class being (row / xcd) % 8, still most expensive first within it
    int      xcd = 0;
    int      tiles_x = 0, tiles_y = 0, frames = 0;
};
struct LearnScratch;         // device scratch (rt_learn.hip)
size_t learn_scratch_bytes(int n);
// Enqueues on stream s: writes d_order (n tile indices, most expensive first),
// d_mask (n lane masks), d_hpix (<= cap heavy pixels, tile * 64 + lane, most
// expensive first) and *d_nhpix (their count).  scratch: learn_scratch_bytes(n).
hipError_t learn_on_device(const LearnParams& lp, const unsigned long long* rec, const unsigned* lane,
                           void* scratch, int* d_order, unsigned long long* d_mask, int* d_hpix, int* d_nhpix,
                           hipStream_t s);

// Kernel launcher (rt_trace.hip).  *kernels (nullable) = the kernels it
// enqueued (2 when the heavy tiles run as a launch of their own).
hipError_t launch_trace(const TraceArgs& a, hipStream_t stream, int* kernels = nullptr);

void set_error(const char* fmt, ...);

// rt_wire.hip: the RGB wire format of the multi-GPU exchange (n_px pixels;
// rgba 16-B aligned, rgb 4-B aligned).
hipError_t wire_pack(const void* rgba, void* rgb, size_t n_px, hipStream_t s);
hipError_t wire_unpack(const void* rgb, void* rgba, size_t n_px, hipStream_t s);

}  // namespace rtamd
