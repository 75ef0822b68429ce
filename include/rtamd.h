/*
 * rtamd.h — C ABI of the MI355X (gfx950) path-trace backend.
 *
 * This is the drop-in boundary for the reference's per-pixel render path
 * (this-Demir/3D-Ray-Tracer-Vulkan).  A Java host binds these symbols through a
 * thin JNI shim; Python binds them through ctypes
 * (3d-ray-tracer-vulkan_amd/rtamd/_lib.py).  Plain C types only: pointers,
 * sizes, and POD structs whose bytes equal the reference's Vulkan buffers.
 *
 * Status convention: every int-returning call returns RT_OK (0) on success and
 * a negative RT_ERR_* code on failure; rt_last_error() then returns a
 * thread-local, human-readable message.  No C++ exception crosses this ABI.
 *
 * Threading: an rt_ctx is single-thread-affine, like the reference's VRT
 * thread (VulkanEngine.java:194-206).  Different contexts may be used from
 * different threads.
 */
#ifndef RTAMD_H
#define RTAMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK               0
#define RT_ERR_INVALID_ARG -1  /* null pointer, bad size, bad dimension        */
#define RT_ERR_NO_DEVICE   -2  /* no gfx950 device / bad device id             */
#define RT_ERR_HIP         -3  /* a HIP runtime call failed                    */
#define RT_ERR_BAD_SCENE   -4  /* node/triangle buffers are malformed          */
#define RT_ERR_NO_SCENE    -5  /* rt_render before rt_upload_scene             */
#define RT_ERR_OOM         -6  /* host or device allocation failed             */
#define RT_ERR_IO          -7  /* file could not be read / parsed              */

/* Byte sizes of the reference's std430/std140 records. */
#define RT_VERTEX_RECORD_BYTES   48  /* one flattened triangle: 3 x (vec3 pos, float pad)  SceneBuilder.java:95-99 */
#define RT_MATERIAL_RECORD_BYTES 16  /* (vec3 albedo, float type)                          SceneBuilder.java:103   */
#define RT_NODE_RECORD_BYTES     48  /* LinearBVHNode, std430                              BVHFlattener.java:19    */
#define RT_CAMERA_UBO_BYTES      80  /* CameraUBO + frameCount + isSkyEnabled              VulkanEngine.java:378-396 */
#define RT_REFERENCE_MAX_BOUNCES 10  /* compute_dynamic_ray.comp:44 */
/* Layout version of the structs below (rt_camera_ubo, rt_stats) and of the
 * calls' argument lists: bumped whenever one changes (round 4 moved
 * rt_stats.pixels to the end, SURVEY.md §8b's order).  A binding compiled
 * against another version must refuse the library (rt_abi_version). */
#define RT_ABI_VERSION 6

typedef struct rt_ctx rt_ctx;

/* Same 80 bytes the reference writes into its camera UBO
 * (VulkanEngine.java:387-395; std140 vec3 at offsets 0/16/32/48; ints at 64/68).
 * frame_count and sky_enabled are accepted and ignored, as in the shader
 * (compute_dynamic_ray.comp:26-34 declares neither). */
typedef struct rt_camera_ubo {
    float   origin[4];
    float   lower_left[4];
    float   horizontal[4];
    float   vertical[4];
    int32_t frame_count;
    int32_t sky_enabled;
    int32_t pad[2];
} rt_camera_ubo;

/* Work counters of one render call, in SURVEY.md §8(b)'s field order.
 * segments = executed iterations of the bounce loop
 * (compute_dynamic_ray.comp:179-232); node_visits = hit_aabb calls (:193);
 * tri_tests = hit_triangle calls (:201); mat_reads = scatter calls (:217).
 * They are counted in the reference's visit order, so they are the same for
 * every implementation of the path.  pixels (after §8(b)'s fields) = the
 * pixels the call traced. */
typedef struct rt_stats {
    uint64_t segments;
    uint64_t node_visits;
    uint64_t tri_tests;
    uint64_t mat_reads;
    double   ms;          /* device time of the trace kernel(s), HIP events */
    uint64_t pixels;
} rt_stats;

/* ---------------------------------------------------------------- engine -- */

/* Replaces VulkanEngine.initVulkan (VulkanEngine.java:211-238).
 * device_ids: HIP ordinals to render on (n_devices >= 1).  With several
 * devices a frame is split into interleaved row bands, one per device, and
 * read back per band.  There is no CPU backend: no gfx950 device is an error. */
int rt_create(const int* device_ids, int n_devices, rt_ctx** out);

/* Replaces VulkanEngine.internalSwapScene (VulkanEngine.java:318-373).
 * vertices : 48 B per flattened triangle (SceneBuilder.java:92-99)
 * materials: 16 B per flattened triangle (SceneBuilder.java:103)
 * bvh_nodes: 48 B per node, preorder, little-endian (BVHFlattener.java:51-97)
 * Deep-copies; the caller may free the buffers on return (the Java host frees
 * them right after upload, VulkanEngine.java:343,351).  Sizes below one record
 * (the reference's 1-float / 1-byte dummies for an empty scene,
 * SceneBuilder.java:61-70) upload an empty scene, which renders sky only.
 * Scenes whose walk records would exceed 4 GB (2^27 - 4 slots of 32 B: about
 * 45M triangles) fail with RT_ERR_BAD_SCENE: the walk addresses its records
 * with 32-bit buffer offsets. */
int rt_upload_scene(rt_ctx* ctx,
                    const void* vertices,  size_t vertex_bytes,
                    const void* materials, size_t material_bytes,
                    const void* bvh_nodes, size_t bvh_bytes);

/* NON-REFERENCE extension (option "extensions" bit 8; the reference scene is
 * triangles only): spheres, 8 floats each
 * (centre.xyz, radius, albedo.rgb, material type 0-3 as the triangle
 * materials), tested after every segment's BVH walk in index order against
 * (T_MIN, closest_t); semantics in oracle/rt_oracle.h ORC_EXT_SPHERES.
 * Deep-copies; n_spheres 0 removes them.  Independent of rt_upload_scene
 * (a scene upload keeps them).  Radii must be finite and > 0, centres finite,
 * n_spheres <= 65536. */
int rt_upload_spheres(rt_ctx* ctx, const float* spheres, int n_spheres);

/* Replaces VulkanEngine.renderFrame (VulkanEngine.java:401-431): renders one
 * width x height frame synchronously and copies it to host memory.
 * out_rgba    : width*height*4 bytes, RGBA8 UNORM, row 0 = top (required)
 * out_radiance: width*height*3 floats, the sqrt'd colour before quantisation
 *               (nullable)
 * stats       : nullable.
 * max_bounces : the shader's MAX_BOUNCES; 10 reproduces the reference. */
int rt_render(rt_ctx* ctx, const rt_camera_ubo* cam,
              int width, int height, int max_bounces,
              uint8_t* out_rgba, float* out_radiance, rt_stats* stats);

/* Device-resident form for multi-GPU tiling and benchmarking: renders the
 * rectangle [x0, x0+tile_w) x [y0, y0+tile_h) of a width x height frame of
 * device 0 of ctx into DEVICE buffers d_out_rgba (tile_w*tile_h*4 B, may be
 * null) and d_out_radiance (tile_w*tile_h*3 floats, may be null), enqueued on
 * `stream` (a hipStream_t of the same HIP runtime; NULL = the null stream).
 * Asynchronous unless stats is non-null, in which case it waits and fills
 * stats.  A process that also uses PyTorch must load torch's HIP runtime
 * first (rtamd/_lib.py does), so that one runtime owns the device pointers. */
int rt_render_tile_device(rt_ctx* ctx, const rt_camera_ubo* cam,
                          int width, int height, int max_bounces,
                          int x0, int y0, int tile_w, int tile_h,
                          void* d_out_rgba, void* d_out_radiance,
                          void* stream, rt_stats* stats);

/* Interleaved row bands, for splitting a frame over GPUs with balanced work:
 * renders every frame row y whose band index y / band_h is congruent to
 * band_off modulo band_stride, packed in increasing y into DEVICE buffers of
 * rt_band_rows(height, band_h, band_stride, band_off) rows of width pixels.
 * Same stream / stats semantics as rt_render_tile_device. */
int rt_render_bands_device(rt_ctx* ctx, const rt_camera_ubo* cam,
                           int width, int height, int max_bounces,
                           int band_h, int band_stride, int band_off,
                           void* d_out_rgba, void* d_out_radiance,
                           void* stream, rt_stats* stats);

/* Row count of such a band set (-1 for bad arguments).  Pure host code. */
int rt_band_rows(int height, int band_h, int band_stride, int band_off);

/* Batched frames over listed row bands, for the multi-GPU frame partitions
 *  and a render loop's frames in flight: ONE launch traces,
 * for each of the n_frames cameras cams[f] (1..16 frames), the frame rows of
 * the band_h-row bands listed in `bands` (n_bands strictly increasing band
 * indices below ceil(height / band_h); a rank's share of a weighted band
 * partition), or the whole frame when bands is NULL.  Frame f's rows are
 * packed in increasing y at rows [f * R, (f + 1) * R) of the DEVICE buffers
 * d_out_rgba (R * width * 4 B per frame, may be null) and d_out_radiance
 * (R * width * 3 floats per frame, may be null), R =
 * rt_band_list_rows(height, band_h, bands, n_bands).  Every pixel is traced
 * exactly as one frame per launch traces it (seed = its global pixel index,
 * compute_dynamic_ray.comp:164); one launch of several frames replaces
 * several small launches, whose per-launch tails and queue slots a rank's
 * share of a frame cannot fill.  The band list is copied to
 * the device once per distinct list.  The accumulation extension takes one
 * frame per launch.  Same stream / stats semantics as rt_render_tile_device
 * (stats: the totals over the frames). */
int rt_render_batch_device(rt_ctx* ctx, const rt_camera_ubo* cams, int n_frames,
                           int width, int height, int max_bounces,
                           int band_h, const int32_t* bands, int n_bands,
                           void* d_out_rgba, void* d_out_radiance,
                           void* stream, rt_stats* stats);

/* Row count of a band list (-1 if the list is not strictly increasing or
 * reaches past the frame).  Pure host code. */
int rt_band_list_rows(int height, int band_h, const int32_t* bands, int n_bands);

/* Batched frames, each over its OWN band list, for the weak-scaling
 * partition that rotates contiguous row pieces over the ranks frame by frame
 * (every rank's launch then holds one whole frame's worth of rows, each piece
 * of a different frame): frame f traces the band_h-row bands
 * bands[f * n_per .. f * n_per + n_per), a strictly increasing list followed
 * by -1 padding only; band_h must divide height.  List position k of frame f is written at rows
 * [f * R + k * band_h, ...) of the DEVICE buffers, R = n_per * band_h =
 * rt_band_lists_rows(height, band_h, bands, n_frames, n_per); padding rows
 * are neither traced nor written.  Otherwise as
 * rt_render_batch_device (stats: totals over the frames' listed rows). */
int rt_render_batch_lists_device(rt_ctx* ctx, const rt_camera_ubo* cams, int n_frames,
                                 int width, int height, int max_bounces,
                                 int band_h, const int32_t* bands, int n_per,
                                 void* d_out_rgba, void* d_out_radiance,
                                 void* stream, rt_stats* stats);

/* R of such lists, n_per * band_h (-1 if a list is bad).  Pure host code. */
int rt_band_lists_rows(int height, int band_h, const int32_t* bands, int n_frames, int n_per);

/* One launch over the same rectangle [x0, x0 + tile_w) x [y0, y0 + tile_h) of
 * n_frames frames (1..16, camera cams[f] each): the tile grid of a multi-GPU
 * frame (rtamd/dist.py TilePlan, BASELINE config 4's 2 x 2 over 4 GPUs) with
 * several frames' tiles per launch, so a rank's launch is a frame's worth of
 * pixels rather than a quarter frame (one quarter-frame launch per frame ran
 * a rank's tiles 3-5x slower per pixel than whole frames: its serial tail,
 * profiles/r06/r6e).  Outputs hold the tiles one after another (n_frames x
 * tile_h x tile_w).  Same stream / stats semantics as rt_render_tile_device. */
int rt_render_batch_rect_device(rt_ctx* ctx, const rt_camera_ubo* cams, int n_frames,
                                int width, int height, int max_bounces,
                                int x0, int y0, int tile_w, int tile_h,
                                void* d_out_rgba, void* d_out_radiance, void* stream, rt_stats* stats);

/* Batched runs of bands, packed: frame f (camera cams[f], 1 <= n_frames <= 16)
 * traces its band_h-row bands [band_lo[f], band_hi[f]) (band_h must divide
 * height; an empty run traces nothing), and its rows follow frame f - 1's in
 * the DEVICE buffers (sum of the runs x band_h rows of width pixels).  The
 * spans partition's launch of two consecutive frames of a rank's span, a run
 * at the span's end merged with its neighbouring whole frame.
 * Otherwise as rt_render_batch_device. */
int rt_render_batch_runs_device(rt_ctx* ctx, const rt_camera_ubo* cams, int n_frames,
                                int width, int height, int max_bounces, int band_h,
                                const int32_t* band_lo, const int32_t* band_hi,
                                void* d_out_rgba, void* d_out_radiance, void* stream, rt_stats* stats);

/* Pipelined frames (overlap the readback with the next
 * frame; the reference waits on a fence after every frame,
 * VulkanEngine.java:410-429).
 *
 * rt_render_async enqueues one whole frame (trace + RGBA8 readback into
 * out_rgba) and returns at once with a ticket; rt_render_wait blocks until that
 * frame is complete in out_rgba.  Option "async_slots" (1..8, default 4) frame
 * slots rotate per device, each tracing on a stream of its own, so with that
 * many frames in flight the frames' traces run at once and every readback
 * overlaps later traces (copies complete in ticket order).  Option
 * "copy_streams" (1 or 2, default 1): 2 splits a one-device frame's readback
 * in two halves on two copy streams (measured slower: 0.40 vs 0.37 ms per
 * frame, profiles/r02/async/copy_streams).
 * The heavy-pixel
 * bar counts the slots as concurrent launches.  Concurrent streams need a
 * hardware queue each, and HIP's default is 4 per process, fixed when the HIP
 * runtime loads: start the host process with GPU_MAX_HW_QUEUES=16 (JVM:
 * `GPU_MAX_HW_QUEUES=16 java ...`; the Python package sets it on import if
 * HIP is not initialised yet); rt_get_option "queues_short" says 1 when the
 * slots cannot each have a queue.
 * out_rgba must stay valid until its ticket completes; it should come from
 * rt_host_alloc (pinned, portable), since a copy into pageable memory cannot run
 * asynchronously.  A Java host wraps rt_host_alloc memory with JNI
 * NewDirectByteBuffer.  Frames are identical to rt_render's. */
void* rt_host_alloc(size_t bytes);
void  rt_host_free(void* p);
int rt_render_async(rt_ctx* ctx, const rt_camera_ubo* cam, int width, int height, int max_bounces,
                    uint8_t* out_rgba, uint64_t* ticket);
int rt_render_wait(rt_ctx* ctx, uint64_t ticket);
/* Non-blocking form of rt_render_wait: *done = 1 when the frame of `ticket`
 * is complete in its out_rgba (rt_render_wait would return at once), else 0.
 * A UI timer (VulkanApp.updateUI, VulkanApp.java:194-235) can poll it instead
 * of blocking its thread. */
int rt_render_poll(rt_ctx* ctx, uint64_t ticket, int* done);

/* Schedule options (no effect on results, which are identical for every
 * setting):
 *   "kernel"        0 only: the one kernel, one lane per pixel (the
 *                   reference's dispatch shape).  The persistent, split and
 *                   tiered kernels (1-3) and the options that tuned them
 *                   (shade_min, blocks_per_cu, seg_limit, heavy_budget,
 *                   prio_after) measured slower and were archived in round 3
 *                   (profiles/r03/archive); setting them is an error.
 *   "walk"          0 = one node per step, 2 = one node per step,
 *                   software-pipelined over compact records: the next node's
 *                   box is requested before this node's triangle test and the
 *                   loop control (default).  Walks 1, 3 (round 4: a leaf in
 *                   two steps), 5, 13, 14 were measured slower and archived.
 *   "accel"         at the next rt_upload_scene: 8 (default) = trace the
 *                   uploaded triangles through a binned-SAH tree built on the
 *                   host (one primitive per reference leaf: the triangle and
 *                   its own leaf box; byte-identical copies dropped), in 8
 *                   preorder layouts, each putting the near child first for
 *                   one octant of ray directions; 1 = one layout (lower child
 *                   first); 0 = the reference's own tree in its DFS order.
 *                   The walk enters a box when t_enter <= closest_t *
 *                   (1 + 2^-10) + 2^-10 and takes a triangle on t < closest_t
 *                   or on a tie with a lower flattened index (the reference's
 *                   first-found); a segment whose hit lies before its own
 *                   box's t_enter is walked again in the reference's order.
 *                   Frames, segments and material reads are the reference
 *                   order's; node visits and triangle tests are the accel
 *                   walk's own.  The exactness argument holds
 *                   when no triangle's rounded t lies more than that margin
 *                   before its own leaf box's t_enter.  Boxes over needle
 *                   triangles (shape class >= 7, where Moeller-Trumbore's t
 *                   error grows) are entered whenever their slab test passes;
 *                   for the rest no tested scene comes within 2^-10 of the
 *                   margin (tests/test_accel_model.py, adversarial slivers,
 *                   grazing rays, far-from-origin meshes), but it is a bound,
 *                   not a proof: accel 0 is the exact mode by construction.  Past the records' slot cap (2^27 - 4
 *                   slots: ~5.6 M triangles at 8 layouts) the upload falls
 *                   back to 1 layout, then to the reference's tree
 *                   ("accel_used").  Heavy tiles / pixels are not split out
 *                   of accel launches (heavy_first still orders the tiles)
 *   "split_bounce"  accel walk, no extensions: b in 1..max_bounces-1 = a
 *                   frame's paths still alive at bounce b leave its kernel for
 *                   the wave's ray slots (packed per wave, no atomics), a scan
 *                   orders them and a second kernel finishes them 64 per wave,
 *                   so the few long late-bounce paths of a tile no longer hold
 *                   a whole wave; 0 (default) = one kernel.
 *                   Same frames; counting and diagnostic launches stay one
 *                   kernel.  Memory: 3 KB of ray slots per wave of a launch
 *                   (64 x 48 B), per launch stream, kept until rt_destroy; a
 *                   launch that would need more than 256 MB (e.g. a batch of
 *                   4K frames) stays one kernel.  Growing a stream's slots
 *                   synchronises that stream
 *   "accel_half"    at the next rt_upload_scene, accel records with the
 *                   internal nodes' boxes in IEEE half precision rounded
 *                   outward (16-B internal records instead of 32; leaves keep
 *                   their exact fp32 boxes and triangles): a walk step of
 *                   internal nodes loads half the bytes, widened boxes are only
 *                   entered more often, so frames are unchanged (DESIGN.md
 *                   §4a).  Forces coop_lanes 0.  0 / 1
 *   "accel_half_used" (rt_get_option only) 1 when device 0's accel records
 *                   are in that format
 *   "accel_wide"    at the next rt_upload_scene, with accel on: 1 = a 4-wide
 *                   tree collapsed from the same SAH tree, one layout of 64-B
 *                   records, children entered in t_enter order with a per-lane
 *                   stack of 12 entries in LDS (accel_build.h format 2; an
 *                   overflow walks the segment in the reference's order).
 *                   Same frames; 0.49x the wave-level loads of the default but
 *                   1.45x its VALU instructions: measured slower (config 3
 *                   1.35x, config 5 1.74x); default 0
 *   "accel_wide_used" (rt_get_option only) 1 if the current scene on device 0
 *                   has format-2 records
 *   "accel_used"    (rt_get_option only) the current scene's layouts on device
 *                   0 (0 = the reference's tree)
 *   "walk_bytes"    (rt_get_option only) bytes of the records one ray walks on
 *                   device 0 (the reference's walk records, or one accel layout)
 *   "coop_lanes"    once at most this many lanes of a wave are still walking,
 *                   the whole wave finishes their walks one ray at a time
 *                   (0..64; 0 = off; -1, the default = 1 on the reference's
 *                   tree, 0 on the accel tree)
 *   "coop_walk"     cooperative walks (the coop tail): 0 = 64-node preorder
 *                   windows (default), 1 = preorder frontier (up to 64 live
 *                   subtrees expanded per round trip)
 *   "coop_window"   the windows' size: 64 or 32 slots; 0 (default) = 32 when
 *                   the scene's walk records exceed 32 MB (the L2s of the 8
 *                   XCDs), else 64
 *   "coop_window_used" (rt_get_option only) the window size the current scene
 *                   gets on device 0
 *   "block_waves"   waves per workgroup, 1 (default: a finished wave frees its
 *                   slot at once) or 4
 *   "heavy_first"   with block_waves 1: 1 (default) = the first
 *                   plain (non-stats) launch of a frame geometry + camera +
 *                   scene runs the diagnostic build, records every wave's
 *                   duration and walk length, and ends with a stream
 *                   synchronisation; later launches with the same key
 *                   dispatch the tiles most expensive first (up to 16 keys
 *                   per device are kept)
 *   "heavy_tiles"   with heavy_first: the first this-many tiles of the order
 *                   are traced one pixel per wave (64 one-wave workgroups per
 *                   tile), every segment walked cooperatively with the
 *                   frontier walk, in a launch of their own.  -1 (default) =
 *                   automatic: the tiles whose walk length exceeds
 *                   "heavy_factor" percent (default 130) of the bulk estimate,
 *                   at most "heavy_cap" percent of one generation of
 *                   one-pixel waves (CUs x 24 / 64 tiles: 96 on MI355X, so 72
 *                   by default), shared by the concurrent launches.  Heavy
 *                   tiles and pixels need coop_lanes > 0 and no extensions
 *                   (and walk 2 for heavy_stream 2); otherwise a launch uses
 *                   the learned order alone
 *   "concurrent_launches" the number of launches of similar work the caller
 *                   keeps in flight on a device at once (1..64, default 1): a
 *                   render loop with two frames in flight says 2, a batch of N
 *                   band offsets traced together says N.  The automatic
 *                   heavy-tile estimate counts a launch's work that many times
 *                   and divides the heavy-tile cap by it.
 *   "heavy_stream"  2 (default) = the heavy tiles' one-pixel workgroups come
 *                   first in the same launch as the other tiles (dispatched in
 *                   index order, so every heavy wave starts at once; one
 *                   launch per frame, no fork / join); 1 = their own launch
 *                   on an auxiliary stream, forked from and joined back to the
 *                   caller's stream, concurrent with the other tiles; 0 = their
 *                   own launch before the other tiles on the caller's stream
 *   "heavy_cap"     automatic heavy tiles / pixels: at most this percentage
 *                   (1..100, default 75) of one generation of one-pixel waves
 *   "heavy_pixels"  with heavy_stream 2 and automatic heavy tiles: 1 (default)
 *                   = split heavy PIXELS, not whole tiles: the learning launch
 *                   also records every pixel's walk length; the pixels whose
 *                   walk exceeds "heavy_pixel_factor" percent (default 50) of
 *                   the bulk estimate are traced one per wave by the first
 *                   workgroups of the launch, and every tile wave skips its
 *                   heavy pixels; 0 = whole heavy tiles
 *   "heavy_pixel_factor" see heavy_pixels (1..100000, default 50)
 *   "reuse_order"   heavy_first: 1 (default) = a camera that has just moved
 *                   (differs from the camera of the last launch with the same
 *                   frame geometry and scene) uses the newest order learned
 *                   for that geometry and scene instead of learning (no
 *                   learning frame while the camera moves; the first repeat of
 *                   a camera learns); 0 = every new camera learns
 *   "heavy_pixels_used" (rt_get_option only) heavy pixels of the last launch
 *   "graph"         plain launches on a non-null stream whose frame is two
 *                   launches (heavy_stream 1): 1 (default) = captured once per
 *                   launch key into a HIP graph and replayed; 0 = launched
 *                   directly.  Counting and learning launches are never
 *                   captured.  Same results.
 *   "learn_cost"    heavy_first order by 1 = wave duration (default) or 0 =
 *                   walk length
 *   "learn_alone"   heavy_first: 1 = a learning launch first waits for the
 *                   device to drain (its wave durations then are not inflated
 *                   by other launches in flight); 0 (default) = it does not
 *   "accel_octants" option accel with 8 layouts: the octant bits (x 1, y 2,
 *                   z 4) that choose a ray's layout; 7 (default) = all three
 *                   (every ray walks near child first on every axis); fewer
 *                   bits touch fewer layouts (half the records with two bits)
 *                   at a worse order on the dropped axes.  Same results.
 *   "xcd_order"     heavy_first, orders learned on the device: 0 (default) =
 *                   the cost order as is; r in 1..4096 = workgroup k, which
 *                   the hardware deals to XCD k % 8, takes from one eighth of
 *                   the tiles: rows of wave tiles in bands of r, every 8th
 *                   band to one eighth (r >= the tile rows: 8 contiguous
 *                   slabs), most expensive first within it, so each XCD's
 *                   L2 serves rays from fewer parts of the scene.  Same
 *                   results.
 *   "order_split"   heavy_first: 0 = every tile in cost order; p in 1..100 =
 *                   only the tiles costing at least p percent of the
 *                   costliest go first (in cost order), the rest keep their
 *                   raster order (frame by frame), which keeps the waves
 *                   running at once on neighbouring tiles
 *   "order_frames"  heavy_first, launches of several frames (the batch entry
 *                   points): 1 = the tiles after the leading ones go row by
 *                   row across the launch's frames (the same image rows of
 *                   every frame run at once); 0 (default) = frame by frame
 *   "heavy_tiles_used" (rt_get_option only) heavy tiles of the last launch
 *   "wave_tile"     pixels per wave (8<<s) x (8>>s), s = 0..3; -1 (default) =
 *                   16x4 on the accel tree (config 3 2% faster than 8x8,
 *                   profiles/r05/r5ac) and when the reference tree's walk
 *                   records exceed 32 MB (config 5: 3% faster), else 8x8 (the
 *                   shader's local_size; config 3 on the reference tree: 0.8%
 *                   faster than 16x4, 6% than 32x2, profiles/r02/tiles)
 *   "wave_tile_used" (rt_get_option only) the tile shape s the current scene
 *                   gets on device 0
 *   "extensions"    NON-REFERENCE features, bits (default 0 = the reference's
 *                   shader exactly):
 *                   1 = honour sky_enabled (@68): a miss is black when it is 0
 *                   2 = a type-3 ("Emissive (Light)") hit ends the path with
 *                       attenuation * albedo (the reference renders it black)
 *                   4 = progressive accumulation: seed += frame_count*W*H
 *                       (frame 0 is the reference's frame), a per-device buffer
 *                       keeps the running sum of the linear colour (frame_count
 *                       0 overwrites it; a new frame partition starts from
 *                       zero) and the output is sqrt(sum / (frame_count+1)).
 *                       The sums are per device, so frames must reach the
 *                       device in frame_count order: rt_render_async
 *                       serialises its slots' traces then; a caller tracing on
 *                       several streams of its own must do the same
 *                   8 = spheres (rt_upload_spheres) after the BVH walk
 *   "async_slots"   rt_render_async frames in flight per device (1..8, default 4)
 *   "copy_streams"  rt_render_async readback copy streams (1 or 2, default 1)
 *   "learn_device"  heavy_first: 1 = learn the order on the device, on the
 *                   learning launch's stream, with no synchronisation (default;
 *                   the default heavy-pixel schedule only); 0 = copy the records
 *                   back and learn on the host after a stream synchronisation
 *   "leaf_align"    at the next rt_upload_scene: 1 = lay the walk records out
 *                   so that no leaf's 64-B record straddles a 128-B line (a
 *                   pad slot before such a leaf); 0 = packed; 2 (default) =
 *                   aligned when the packed records exceed 32 MB (the L2s of
 *                   the 8 XCDs), else packed
 *   "leaf_align_used" (rt_get_option only) 1 if the current scene's records
 *                   on device 0 hold pad slots
 *   "plain_kernels" (rt_get_option only) production-build trace kernels enqueued
 *                   on device 0 so far (not counting, diagnostic or learning
 *                   launches): lets a profiler's kernel trace be cut at a
 *                   caller's region (bench.py, tools/rocprof_union.py)
 *   "hw_queues"     (rt_get_option only) GPU_MAX_HW_QUEUES as seen by rt_create
 *                   (4, HIP's default, when unset)
 *   "queues_short"  (rt_get_option only) 1 when async_slots + 2 > hw_queues:
 *                   the slots' traces then share hardware queues and run one
 *                   after another (set GPU_MAX_HW_QUEUES before the process
 *                   initialises HIP)
 * Defaults can also be set with the environment variables RTAMD_ACCEL, RTAMD_ACCEL_HALF,
 * RTAMD_OPTS ("name=value,..." of any option above), RTAMD_WALK, RTAMD_COOP_LANES, RTAMD_COOP_WALK, RTAMD_BLOCK_WAVES, RTAMD_HEAVY_FIRST,
 * RTAMD_HEAVY_TILES, RTAMD_HEAVY_FACTOR, RTAMD_HEAVY_STREAM (0 / 1 / 2),
 * RTAMD_HEAVY_PIXELS, RTAMD_LEARN_COST and RTAMD_GRAPH. */
int rt_set_option(rt_ctx* ctx, const char* name, int64_t value);
/* Diagnostics: with option "diag" = 1, the kernel records per wave
 * 8 words: {start, end} (s_memrealtime, 100 MHz), {XCC id << 32 | HW_ID},
 * {block << 8 | wave}, {lockstep walk iterations}, {cooperative windows},
 * {ticks spent in the cooperative tail}, {the lanes' own lockstep steps,
 * summed over the wave} into a device buffer (a heavy pixel's one-pixel wave
 * leaves words 4-7 zero; lane utilisation of the lockstep walk = sum of word 7
 * / (64 x sum of word 4));
 * rt_diag_copy copies up to cap_words 64-bit words of the last launch
 * (n_words = words recorded).  Not for timing runs. */
int rt_diag_copy(rt_ctx* ctx, void* dst, size_t cap_words, size_t* n_words);
int rt_get_option(rt_ctx* ctx, const char* name, int64_t* value);

/* Replaces VulkanEngine.cleanup. Null is accepted. */
int rt_destroy(rt_ctx* ctx);

/* Thread-local message for the last failing call on this thread. */
const char* rt_last_error(void);

/* RT_ABI_VERSION of the library, and sizeof(rt_stats) / sizeof(rt_camera_ubo)
 * as it was compiled (nullable): a host checks them once after loading. */
int rt_abi_version(size_t* stats_bytes, size_t* camera_bytes);

/* The build's provenance: "src=<16 hex> git=<12 hex>", the first 16 hex digits
 * of SHA-256 over the library's sources and headers concatenated in the
 * Makefile's order (SRC_ALL), and the checkout's HEAD when it was built.  The
 * same string is embedded in the file after "RTAMD_BUILD_ID:", so a test can
 * check a library against the tree without loading it (rtamd/_lib.py
 * source_hash, tests/conftest.py, __graft_entry__.smoke). */
const char* rt_build_id(void);

/* Node / triangle counts and tree depth of the uploaded scene. */
int rt_scene_info(rt_ctx* ctx, size_t* n_nodes, size_t* n_tris, int* max_depth);

/* The validation rt_upload_scene performs, without a device (pure host code):
 * RT_OK, or RT_ERR_BAD_SCENE with the reason in rt_last_error().  The node
 * array must be the reference flattener's preorder layout (left child i+1,
 * BVHFlattener.java:51-75) with every leaf's triangle inside the vertex and
 * material buffers.  n_nodes receives the nodes reachable from the root. */
int rt_scene_validate(const void* vertices, size_t vertex_bytes,
                      const void* materials, size_t material_bytes,
                      const void* bvh_nodes, size_t bvh_bytes,
                      size_t* n_nodes, int* max_depth);

/* Option "accel"'s records, built on the host exactly as
 * rt_upload_scene builds them for a context with accel on (pure host code, no
 * device): the binned-SAH tree over the reference leaves' (triangle, box)
 * pairs, n_layouts (1, or 8 = one per ray-direction octant) near-first
 * preorder layouts in the walk-record format, 8 32-bit words per 32-B slot;
 * n_layouts | RT_ACCEL_FORMAT_HALF: option accel_half's format, 4 words per
 * 16-B slot, internal boxes in half precision rounded outward;
 * n_layouts | RT_ACCEL_FORMAT_WIDE: option accel_wide's 4-wide tree, one
 * layout of 64-B records (16 words; "slots" = records).
 * Writes up to cap_words words (out_words may be NULL to size the call) and
 * *n_words = the words of the records (n_layouts * slots, + 64 B of padding);
 * info (nullable) receives {n_layouts, slots per layout, root is a leaf,
 * primitives after dropping byte-identical duplicates, reference leaves, tree
 * depth, the largest shape class, primitives of class >= 7 (thin: their
 * boxes are entered whenever their slab test passes, "accel" above)}.  Only the root's subtree counts (nodes past the root's skip are
 * never visited by the reference).  The capacity fallback of rt_upload_scene
 * applies: 8 layouts past the slot cap are built as 1 (info[0] = 1), and a
 * scene too large for one layout gets no records (RT_OK, *n_words = 0, info
 * all 0: rt_upload_scene walks the reference's own tree).  An analysis and
 * test entry point (oracle/rt_accel_model.c walks these records on the CPU);
 * a host embedding the backend never needs it. */
/* The multi-GPU wire format (rtamd/dist.py span_send / span_finish_recvs,
 * DESIGN.md §6): a frame's alpha byte is always 255 (compute_dynamic_ray.comp:235),
 * so rows cross the xGMI links as RGB.  rt_pack_rgb packs n_px RGBA8 pixels
 * of d_rgba into 3-byte RGB at d_rgb; rt_unpack_rgb writes n_px RGB pixels
 * back as RGBA8 with alpha 255.  Device pointers on the stream's device; d_rgba
 * 16-B aligned, d_rgb 4-B aligned; enqueued on `stream`, no synchronisation. */
int rt_pack_rgb(const void* d_rgba, void* d_rgb, size_t n_px, void* stream);
int rt_unpack_rgb(const void* d_rgb, void* d_rgba, size_t n_px, void* stream);

#define RT_ACCEL_FORMAT_HALF 0x100
#define RT_ACCEL_FORMAT_WIDE 0x200
int rt_accel_records(const void* vertices, size_t vertex_bytes,
                     const void* materials, size_t material_bytes,
                     const void* bvh_nodes, size_t bvh_bytes, int n_layouts,
                     uint32_t* out_words, size_t cap_words, size_t* n_words, int32_t info[8]);

/* ----------------------------------------------------------- scene build -- */
/* Host-side producers of the three buffers, replacing the Java SceneBuilder
 * (SceneBuilder.java:38-118), BVHBuilder (BVHBuilder.java:48-108), BVHFlattener
 * (BVHFlattener.java:30-97) and Camera (Camera.java:44-68).  Pure CPU code. */

/* Node / flattened-triangle counts the reference builder produces for n input
 * triangles (they depend on n only: a range of 1 or 2 triangles becomes one
 * node with two leaves, BVHBuilder.java:60-71). */
int rt_bvh_layout_size(size_t n_tris, size_t* n_nodes, size_t* n_flat_tris);

/* Builds the median-split BVH and writes the three reference buffers.
 * tri_verts : n_tris*9 doubles, post-transform vertices v0,v1,v2 (Triangle.java:35-51)
 * tri_mats  : n_tris*4 floats, (r,g,b,type) per triangle
 * axis_seed : seeds the per-node split axis (the reference's is unseeded,
 *             BVHBuilder.java:53; pixels do not depend on it)
 * out_vertices : n_flat*12 floats; out_materials: n_flat*4 floats;
 * out_nodes    : n_nodes*48 bytes. Sizes from rt_bvh_layout_size.
 * n_threads    : 0 = all hardware threads.  Output does not depend on it. */
int rt_build_scene(const double* tri_verts, const float* tri_mats, size_t n_tris,
                   uint64_t axis_seed, int n_threads,
                   float* out_vertices, float* out_materials, void* out_nodes);

/* Camera.recalculateViewport (Camera.java:44-68) in double, cast to float as
 * Vec3.store does (Vec3.java:132-136). */
int rt_camera_from_lookat(const double origin[3], const double lookat[3],
                          const double vup[3], double vfov_deg, double aspect,
                          rt_camera_ubo* out);

/* OBJ mesh (SceneBuilder.loadModel, SceneBuilder.java:129-191), read the way
 * the reference's Assimp call (aiImportFile(path, aiProcess_Triangulate |
 * aiProcess_JoinIdenticalVertices), :144) reads it: numbers by Assimp's
 * fast_atof (not a correctly rounded strtof), 'v' lines of 3, 4 (/w) or 6
 * components; a quad is split along the diagonal from its concave corner, or
 * from corner 0 when convex; a larger polygon is projected along its Newell
 * normal and ear-clipped (TriangulateProcess).  Faces of 1-2 indices are
 * skipped, as the Java loop skips them.  Triangles in file order.  Restated
 * from Assimp's published sources (csrc/scene_build.cpp, independently in
 * oracle/obj_oracle.py); parity vs a real Assimp run is unpinned. */
typedef struct rt_mesh rt_mesh;
int    rt_mesh_load_obj(const char* path, rt_mesh** out);
size_t rt_mesh_tri_count(const rt_mesh* mesh);
/* Writes tri_count*9 doubles: float(obj) * scale + position, in double
 * (SceneBuilder.java:172-174). */
int    rt_mesh_transform(const rt_mesh* mesh, const double scale[3],
                         const double position[3], double* out_tri_verts);
int    rt_mesh_free(rt_mesh* mesh);

/* Seeded procedural closed mesh (a displaced ellipsoid shell) with exactly
 * n_tris triangles (n_tris even, >= 8) filling the box [bmin, bmax]; used for
 * the synthetic 50k / 1M triangle configurations. */
int rt_mesh_procedural(size_t n_tris, uint64_t seed,
                       const double bmin[3], const double bmax[3],
                       double* out_tri_verts);

#ifdef __cplusplus
}
#endif
#endif /* RTAMD_H */
