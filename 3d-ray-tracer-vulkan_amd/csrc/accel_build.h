// accel_build.h — the runtime-built acceleration structure of option "accel"
// (pure host C++; no HIP types, so tools/accel_study builds it with g++).
//
// The reference's BVH is a median split on a random axis, visited left child
// first (BVHBuilder.java:48-93, compute_dynamic_ray.comp:185-210).  Its tree
// is random on every build (BVHBuilder.java:53, an unseeded ThreadLocalRandom),
// so its frame is a function of the triangles, not of the tree, except on
// floating-point ties.  Option accel traces the same triangles through a
// binned-SAH tree built here from the uploaded buffers, visited near child
// first, with the two rules that make the closest hit the reference's
// (DESIGN.md §4a):
//   * a box is entered when t_enter <= closest_t (the reference: <), so a
//     triangle whose t equals closest_t is still tested;
//   * a triangle hit is taken when t < closest_t, or t == closest_t and its
//     flattened index is lower than the current hit's: the reference visits
//     leaves in preorder, which is flattened-index order, and keeps the first
//     hit found at a given t (:122, strict <).
// Every leaf keeps its triangle's own box from the reference's leaf node (the
// box the reference tests before the triangle), so a triangle is tested only
// where the reference could test it.
//
// Records: the walk-2 slot format of rt_internal.h (DevScene::walk), packed
// (no pad slots): an internal node one 32-B slot, a leaf two (box, then its
// triangle v0 / e1 / e2).  Bit 29 of word 3 (kAccelForce) marks a record whose
// subtree holds a thin triangle (shape class >= kAccelClassMin; a leaf: its
// own): the walk enters it whenever its slab test passes, whatever closest_t,
// and every other record with the 2^-10 margin.  An internal node's word 7 is
// L(first child) << 31 (the reference's walk records keep it in bit 0).  n_layouts copies of the tree in preorder, each with
// its own child order: layout o puts first, at a node split on axis a, the
// child on the side a ray with sign bit ((o >> a) & 1) on axis a reaches first
// (n_layouts 1: always the lower child).  A ray walks the layout of its
// direction's octant (sign bits of d.x, d.y, d.z), so the stackless skip walk
// is a near-first ordered traversal.
//
// Format 1 ("half", option accel_half): 16-B slots (no room for R: every
// internal node takes the tree's largest, relax_max).  An internal node is one
// slot: its box in IEEE half precision rounded outward (lo down, hi up; words
// 0-2 = lo.x | lo.y << 16, lo.z | hi.x << 16, hi.y | hi.z << 16) and word 3 =
// skip | L(first child) << 30 | L(skip) << 31.  A leaf is four slots, the same
// 64 bytes as format 0's two (its exact fp32 box, triangle index, v0 / e1 /
// e2).  A subtree of m triangles takes 5m - 1 slots; a walk step of internal
// nodes loads 16 B instead of 32.  Widened internal boxes are only entered
// more often: every leaf box and triangle test is format 0's.
//
// Format 2 ("wide", option accel_wide): a 4-wide tree collapsed from the same
// SAH tree (each wide node takes its binary node's children, the
// largest-area internal one split until there are four), one layout, 64-B
// records of which a step reads 48 B (3 loads); a ray orders the children it
// enters by t_enter and keeps the rest on a short per-lane stack.  A wide
// node: words 0-2 its box's lo (the quantisation origin), word 3 = the
// exponents e_x, e_y, e_z (int8, bytes 0-2) | child count (2-4) << 24; words
// 4-9 the children's boxes on the grid origin + q 2^e, 8 bits per bound, byte
// i = child i (lo.x, lo.y, lo.z, hi.x, hi.y, hi.z), every bound rounded
// outward in the kernel's own float arithmetic; word 10 = the children's
// first record (they are one contiguous block) | the node's largest shape
// class << 27 (its margin factor, accel_relax); word 11 = byte i: child i's
// flags (1: a leaf, 2: a thin leaf, entered whenever its slab test passes, 4:
// a subtree of class >= 7, tested with the node's factor).  A leaf: word 0 =
// triangle index | thin << 29 | 1 << 30; words 1-3 v0, 4-6 e1, 8-10 e2 (the
// triangle test's 48 bytes, with lo.x in word 7 and lo.y in word 11); words
// 12-15 lo.z, hi.xyz: the rest of the exact box, read only when the triangle
// test finds a hit the walk would take.  Record 0 is the root.
#pragma once
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rtamd {

struct AccelHost {
    std::vector<uint32_t> rec;      // 8 words per slot (format 1: 4, format 2: 16), n_layouts * slots slots, + 64 B of zero
                                    //   padding
    int format = 0;                 // 0: 32-B slots, fp32 boxes; 1: 16-B slots, half-precision internal boxes;
                                    //   2: 64-B records of the 4-wide tree (slots = records)
    int n_layouts = 0;              // 1 or 8
    int slots = 0;                  // slots per layout (0: empty scene)
    int root_leaf = 0;              // the root is a leaf (a one-triangle scene)
    int n_prims = 0;                // leaves: triangles after removing exact duplicates
    int n_inputs = 0;               // leaves of the reference tree
    int depth = 0;                  // deepest leaf (root = 0)
    double sah = 0.0;               // SAH cost of the tree (internal 1, leaf 1, relative to the root box area)
    int max_class = 0;              // the largest shape class (accel_class) of the primitives
    int n_thin = 0;                 // primitives of class >= kAccelClassMin
    float relax_max = 0.0f;         // accel_relax(max_class): format 1's margin for every internal node
};

// The shape class of a triangle, floor(-log2 sin(angle at v0)) in 0..31
// (31: degenerate), sin = |e1 x e2| / (|e1| |e2|) in double from the float
// edges hit_triangle computes (compute_dynamic_ray.comp:106-107).  Moeller-
// Trumbore's t carries a relative error that grows as 1 / sin: the audit of
// tools/accel_adversarial.py measured hits on needle triangles of class 16
// whose rounded t lay 17 margins (2^-10 relative) before their own box's
// t_enter, the case in which the accel walk could miss the reference's hit.
constexpr int kAccelClassMin = 7;
int accel_class(const float e1[3], const float e2[3]);
// The margin factor R a box whose subtree's largest class is cls needs: the
// walk must enter it when t_enter <= closest_t * R + 2^-10.  Class < 7: 1 +
// 2^-10; else 1 + 2^(cls - 16) (class 16: 2, class 31: 32769), growing as the
// t error does, 64x the error measured at class 16 (the audit's bound,
// oracle/rt_accel_model.c).  Format 0 applies 1 + 2^-10 below class 7 and
// enters a record of class >= 7 whenever its slab test passes (kAccelForce:
// R = infinity, one bit test in the walk instead of a per-record factor);
// format 1 applies accel_relax(max_class) at every internal node, format 2 the
// node's own class.
float accel_relax(int cls);
// Format 0: bit 29 of a record's word 3, a subtree of class >= kAccelClassMin
// (internal skips and triangle indices stay below 2^29).
constexpr uint32_t kAccelForce = 1u << 29;

// The layouts do not fit the slot cap (accel_build's return value).
constexpr int kAccelTooBig = -2;
// Format 2's record cap: 64-B records addressed by 32-bit buffer offsets.
constexpr int64_t kWideCap = (int64_t)(1u << 26) - 2;
// The per-lane stack of the wide walk (entries), and the decode of format 2's
// grid (accel_build.cpp; the kernel and oracle/rt_accel_model.c restate it).
constexpr int kWideStack = 12;
float wide_decode(float origin, int q, int e);

// Builds the records from the reference's buffers (the rt_upload_scene
// inputs: 48-B vertex records, 16-B materials, 48-B preorder nodes).  The
// buffers must already have passed build_host_scene's validation, and
// bvh_bytes must cover only the nodes the root's subtree holds (HostScene::end
// x 48): a node past the root's skip is never visited by the reference's DFS
// (compute_dynamic_ray.comp:185-210), so its leaf is not a primitive.  Returns
// 0, kAccelTooBig when n_layouts copies exceed the slot cap (the 32-bit buffer
// offsets: 2^27 - 4 slots, ~5.6 M triangles at 8 layouts; cap_slots > 0 lowers
// it, for tests), or -1 with *err set.  n_threads: 0 = hardware concurrency.
// format: 0 or 1 (above).
int accel_build(const void* vertices, size_t vertex_bytes, const void* materials, size_t material_bytes,
                const void* bvh_nodes, size_t bvh_bytes, int n_layouts, int n_threads, AccelHost* out,
                std::string* err, int format = 0, int64_t cap_slots = 0);

// accel_build with the capacity fallback: n_layouts 8 that do not fit become
// 1 layout (out->n_layouts says which).  Returns 0, kAccelTooBig when one
// layout does not fit either (the caller then walks the reference's own
// tree, option accel 0, whose records reach ~45 M triangles), or -1.
int accel_build_fit(const void* vertices, size_t vertex_bytes, const void* materials, size_t material_bytes,
                    const void* bvh_nodes, size_t bvh_bytes, int n_layouts, AccelHost* out, std::string* err,
                    int format = 0, int64_t cap_slots = 0);

// Half-precision bits of the largest half <= x (-inf below -65504), and of the
// smallest half >= x: the outward rounding of format 1's internal boxes.
uint16_t half_bits_down(float x);
inline uint16_t half_bits_up(float x) { return (uint16_t)(half_bits_down(-x) ^ 0x8000u); }

// The layout a ray with direction d walks: its octant (sign bits) when
// n_layouts is 8, else 0.
inline int accel_layout(float dx, float dy, float dz, int n_layouts) {
    if (n_layouts != 8) return 0;
    return (std::signbit(dx) ? 1 : 0) | (std::signbit(dy) ? 2 : 0) | (std::signbit(dz) ? 4 : 0);
}

}  // namespace rtamd
