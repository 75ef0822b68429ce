// fast_bvh.h — the second acceleration structure of the certified traversal
// (DESIGN.md §4b): a binned-SAH BVH2 over the reference's leaf triangles,
// built once per rt_upload_scene next to the reference's own preorder nodes.
//
// Why a second BVH.  The reference's result is fixed by its stack DFS over its
// median-split, random-axis tree (compute_dynamic_ray.comp:185-210).  That walk
// is exact but long: a few rays visit thousands of nodes and set the frame time.
// The certified walk instead finds the lexicographic minimum (t, leaf preorder
// index) over every triangle that passes hit_triangle's tests (:105-129), front
// to back over this BVH, and then proves, with one box test on the winner's own
// reference leaf, that the reference DFS would have returned the same triangle
// and the same closest_t (the theorem in DESIGN.md §4b).  Culling here is
// conservative with respect to the float Möller–Trumbore arithmetic: every
// child carries margin constants from a forward error bound of that
// arithmetic, so no triangle that the reference could report is ever culled.
//
// Everything here is host code (plain C++), shared by rt_upload_scene and by
// the analysis tool tools/fastpath_sim.cpp.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rtamd {
namespace fast {

// One deduplicated triangle: the exact operands hit_triangle uses
// (v0, e1 = v1 - v0, e2 = v2 - v0 in binary32, :106-107), the flattened
// triangle index the reference records as the hit (:199), and the preorder
// index of its reference leaf node (the tie-break and the certificate box).
struct Tri {
    float v0[3], e1[3], e2[3];
    int32_t tri;
    int32_t leaf;
};

// One child as its parent sees it.
//   lo/hi        box of the child's triangles (their float vertices)
//   axis, ca, sa normal cone: every triangle normal line lies within the angle
//                alpha (cos ca, sin sa) of the axis line
//   a2min        min |e1 x e2| over the child's triangles
//   emax         max(|e1|_2, |e2|_2) over the child's triangles
// The walk turns these, per ray, into a lower bound on |det| and from it into
// the margins of the conservative box test (margins() below).
struct ChildBox {
    float lo[3], hi[3];
    float axis[3], ca, sa;
    float a2min, emax;
};

// Margins of one child for one ray (the forward error bound of hit_triangle,
// DESIGN.md §4b).  S2 bounds |o - v|_2 and Sinf |o - v|_inf over the child's
// vertices; dabs = |d . axis|.  Returns false when no bound holds (the child
// is then never culled).  Otherwise r inflates the box and m is subtracted
// from its t_enter before the compare with closest_t.
struct MarginConsts {
    float kdet;     // |delta det| <= kdet * emax^2, |delta num| <= kdet * S2 * emax (^2)
    float g2, g3;   // gamma_2, gamma_3
    float ulscene;  // 1.01 u Lscene
};

// Child references: >= 0 an internal node; < 0 a leaf range of tris[].
inline int32_t make_leaf(int first, int count) { return ~(int32_t)((uint32_t)first | ((uint32_t)(count - 1) << 28)); }
inline int leaf_first(int32_t c) { return (int)((uint32_t)~c & 0x0FFFFFFFu); }
inline int leaf_count(int32_t c) { return (int)((uint32_t)~c >> 28) + 1; }
constexpr int kLeafMaxLimit = 8;

struct Node {
    ChildBox c[2];
    int32_t child[2];
};

struct BuildParams {
    int leaf_max = 1;          // triangles per leaf (1..8)
    int bins = 32;             // SAH bins per axis
    int orient_classes = 0;    // experimental: split the top by normal direction (0, 3 or 13 classes)
};

struct Bvh {
    std::vector<Node> nodes;   // nodes[0] is the root (absent for an empty scene)
    std::vector<Tri> tris;
    float root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};
    float lscene = 0.f;        // max |coordinate| over all vertices
    int depth = 0;
    MarginConsts mc{};
    int n_ref_leaves = 0;
    // The certificate needs the reference's boxes to nest (child inside
    // parent) and to be strictly positive in extent; when they
    // are not, the scene keeps the exact reference walk only.
    bool certifiable = false;
    std::string why_not;
};

// Builds the fast BVH from the reference's buffers (48-B vertex records,
// 48-B preorder nodes; already validated by build_host_scene).  Returns 0, or
// -1 with *err on malformed input.
int build_fast_bvh(const void* vertices, size_t vertex_bytes, const void* bvh_nodes, size_t bvh_bytes,
                   const BuildParams& p, Bvh* out, std::string* err);

}  // namespace fast
}  // namespace rtamd
