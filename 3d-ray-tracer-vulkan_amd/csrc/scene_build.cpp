// scene_build.cpp — host producers of the three scene buffers and the camera
// UBO (pure CPU C++, no HIP).  Restates, for a host without Java:
//   SceneBuilder.buildScene / loadModel   SceneBuilder.java:38-191
//   BVHBuilder.buildRecursive + comparator BVHBuilder.java:48-108
//   BVHFlattener.flattenRecursive          BVHFlattener.java:51-97
//   Triangle.calculateBoundingBox          Triangle.java:61-71
//   AABB.surroundingBox                    AABB.java:38-46
//   Camera.recalculateViewport             Camera.java:44-68
// All geometry is double until the float casts the Java code makes.
//
// Determinism: the split axis of the node with preorder index k is a hash of
// (axis_seed, k) instead of ThreadLocalRandom (BVHBuilder.java:53), so the
// buffers are reproducible and subtrees can be built on several threads with
// byte-identical output.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <string>
#include <strings.h>
#include <thread>
#include <vector>

#include "../../include/rtamd.h"

namespace rtamd {
void set_error(const char* fmt, ...);
}
using rtamd::set_error;

namespace {

// ---------------------------------------------------------- Java semantics --

// java.lang.Math.min / max for doubles: NaN wins, -0.0 < +0.0.
inline double jmin(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0) return std::signbit(a) ? a : b;
    return a <= b ? a : b;
}
inline double jmax(double a, double b) {
    if (a != a) return a;
    if (a == 0.0 && b == 0.0) return std::signbit(a) ? b : a;
    return a >= b ? a : b;
}

// Double.compare as a signed 64-bit key (NaNs canonical and largest,
// -0.0 < +0.0), so comparisons are integer compares.
inline int64_t dkey(double d) {
    int64_t b;
    if (d != d) d = std::numeric_limits<double>::quiet_NaN();
    std::memcpy(&b, &d, 8);
    if (d != d) b = 0x7ff8000000000000LL;   // Double.doubleToLongBits canonical NaN
    return b < 0 ? (b ^ 0x7fffffffffffffffLL) : b;
}

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// Split axis of the internal node with preorder index k (0 = x, 1 = y, 2 = z).
inline int split_axis(uint64_t seed, uint64_t k) {
    return (int)((splitmix64(seed ^ (k * 0xD1B54A32D192ED03ULL)) >> 32) % 3u);
}

struct Box { double mn[3], mx[3]; };

inline Box surround(const Box& a, const Box& b) {   // AABB.surroundingBox
    Box r;
    for (int k = 0; k < 3; ++k) {
        r.mn[k] = jmin(a.mn[k], b.mn[k]);
        r.mx[k] = jmax(a.mx[k], b.mx[k]);
    }
    return r;
}

// Node / leaf counts for a range of n triangles (BVHBuilder.java:60-78).
size_t nodes_for(size_t n) {
    if (n == 0) return 0;
    if (n <= 2) return 3;
    return 1 + nodes_for(n / 2) + nodes_for(n - n / 2);
}
size_t leaves_for(size_t n) {
    if (n == 0) return 0;
    if (n <= 2) return 2;
    return leaves_for(n / 2) + leaves_for(n - n / 2);
}

struct Builder {
    const double* verts;        // n*9
    const float*  mats;         // n*4
    uint64_t      seed;
    std::vector<Box> tri_box;   // Triangle.calculateBoundingBox
    std::vector<int64_t> key[3];// centroid keys per axis
    std::vector<uint32_t> order;
    float* out_v;
    float* out_m;
    unsigned char* out_n;
    int max_par_depth;

    void write_node(size_t idx, const Box& b, int32_t data, int32_t count) {
        unsigned char* r = out_n + idx * RT_NODE_RECORD_BYTES;
        float f[8] = {(float)b.mn[0], (float)b.mn[1], (float)b.mn[2], 0.0f,
                      (float)b.mx[0], (float)b.mx[1], (float)b.mx[2], 0.0f};
        std::memcpy(r, f, 32);
        std::memcpy(r + 32, &data, 4);
        std::memcpy(r + 36, &count, 4);
        std::memset(r + 40, 0, 8);
    }

    // Leaf = one Triangle in the flattened order (BVHFlattener.java:85-95,
    // SceneBuilder.java:95-103).
    void write_leaf(size_t node_idx, size_t flat_idx, uint32_t tri) {
        write_node(node_idx, tri_box[tri], (int32_t)(-(int64_t)flat_idx - 1), -1);
        const double* v = verts + (size_t)tri * 9;
        float* o = out_v + flat_idx * 12;
        for (int k = 0; k < 3; ++k) {
            o[4 * k + 0] = (float)v[3 * k + 0];
            o[4 * k + 1] = (float)v[3 * k + 1];
            o[4 * k + 2] = (float)v[3 * k + 2];
            o[4 * k + 3] = 0.0f;
        }
        std::memcpy(out_m + flat_idx * 4, mats + (size_t)tri * 4, 16);
    }

    // buildRecursive(objects, start, end) + flattenRecursive of the node it
    // returns: node_idx = its preorder index, leaf0 = flattened index of its
    // first leaf.
    Box build(size_t start, size_t end, size_t node_idx, size_t leaf0, int depth) {
        const size_t n = end - start;
        const int axis = split_axis(seed, node_idx);
        if (n == 1) {                                  // left = right = objects[start]
            const uint32_t t = order[start];
            write_leaf(node_idx + 1, leaf0, t);
            write_leaf(node_idx + 2, leaf0 + 1, t);
            const Box b = surround(tri_box[t], tri_box[t]);
            write_node(node_idx, b, (int32_t)(node_idx + 1), (int32_t)(node_idx + 2));
            return b;
        }
        if (n == 2) {
            uint32_t a = order[start], c = order[start + 1];
            if (!(key[axis][a] < key[axis][c])) std::swap(a, c);   // compare(a, b) < 0 keeps order
            write_leaf(node_idx + 1, leaf0, a);
            write_leaf(node_idx + 2, leaf0 + 1, c);
            const Box b = surround(tri_box[a], tri_box[c]);
            write_node(node_idx, b, (int32_t)(node_idx + 1), (int32_t)(node_idx + 2));
            return b;
        }
        const std::vector<int64_t>& ka = key[axis];
        std::stable_sort(order.begin() + start, order.begin() + end,
                         [&ka](uint32_t x, uint32_t y) { return ka[x] < ka[y]; });
        const size_t mid = start + n / 2;
        const size_t left_idx = node_idx + 1;
        const size_t right_idx = left_idx + nodes_for(mid - start);
        const size_t right_leaf0 = leaf0 + leaves_for(mid - start);
        Box bl, br;
        if (depth < max_par_depth && n >= 32768) {
            std::thread th([&] { bl = build(start, mid, left_idx, leaf0, depth + 1); });
            br = build(mid, end, right_idx, right_leaf0, depth + 1);
            th.join();
        } else {
            bl = build(start, mid, left_idx, leaf0, depth + 1);
            br = build(mid, end, right_idx, right_leaf0, depth + 1);
        }
        const Box b = surround(bl, br);
        write_node(node_idx, b, (int32_t)left_idx, (int32_t)right_idx);
        return b;
    }
};

}  // namespace

extern "C" {

int rt_bvh_layout_size(size_t n_tris, size_t* n_nodes, size_t* n_flat_tris) {
    if (!n_nodes || !n_flat_tris) { set_error("rt_bvh_layout_size: null output"); return RT_ERR_INVALID_ARG; }
    if (n_tris > (size_t)1 << 29) { set_error("rt_bvh_layout_size: too many triangles"); return RT_ERR_INVALID_ARG; }
    *n_nodes = nodes_for(n_tris);
    *n_flat_tris = leaves_for(n_tris);
    return RT_OK;
}

int rt_build_scene(const double* tri_verts, const float* tri_mats, size_t n_tris,
                   uint64_t axis_seed, int n_threads,
                   float* out_vertices, float* out_materials, void* out_nodes) {
    if (n_tris == 0) return RT_OK;
    if (!tri_verts || !tri_mats || !out_vertices || !out_materials || !out_nodes) {
        set_error("rt_build_scene: null pointer");
        return RT_ERR_INVALID_ARG;
    }
    if (n_tris > (size_t)1 << 29) { set_error("rt_build_scene: too many triangles"); return RT_ERR_INVALID_ARG; }
    try {
        Builder b;
        b.verts = tri_verts;
        b.mats = tri_mats;
        b.seed = axis_seed;
        b.out_v = out_vertices;
        b.out_m = out_materials;
        b.out_n = static_cast<unsigned char*>(out_nodes);
        unsigned hw = n_threads > 0 ? (unsigned)n_threads : std::max(1u, std::thread::hardware_concurrency());
        int pd = 0;
        while ((1u << pd) < hw && pd < 8) ++pd;
        b.max_par_depth = pd;
        b.tri_box.resize(n_tris);
        for (int a = 0; a < 3; ++a) b.key[a].resize(n_tris);
        b.order.resize(n_tris);
        const double eps = 0.0001;                 // Triangle.java:65
        for (size_t t = 0; t < n_tris; ++t) {
            const double* v = tri_verts + t * 9;
            Box& bx = b.tri_box[t];
            for (int k = 0; k < 3; ++k) {
                bx.mn[k] = jmin(v[k], jmin(v[3 + k], v[6 + k]));
                bx.mx[k] = jmax(v[k], jmax(v[3 + k], v[6 + k]));
            }
            // max = max.add(new Vec3(eps,0,0)) etc.: each add touches all
            // three components (x + 0.0 turns -0.0 into +0.0).
            for (int k = 0; k < 3; ++k) {
                if (bx.mx[k] - bx.mn[k] < eps) {
                    for (int j = 0; j < 3; ++j) bx.mx[j] = bx.mx[j] + (j == k ? eps : 0.0);
                }
            }
            for (int a = 0; a < 3; ++a) b.key[a][t] = dkey((bx.mn[a] + bx.mx[a]) / 2.0);
            b.order[t] = (uint32_t)t;
        }
        b.build(0, n_tris, 0, 0, 0);
    } catch (const std::bad_alloc&) {
        set_error("rt_build_scene: out of memory");
        return RT_ERR_OOM;
    } catch (const std::exception& e) {
        set_error("rt_build_scene: %s", e.what());
        return RT_ERR_INVALID_ARG;
    }
    return RT_OK;
}

int rt_camera_from_lookat(const double origin[3], const double lookat[3], const double vup[3],
                          double vfov_deg, double aspect, rt_camera_ubo* out) {
    if (!origin || !lookat || !vup || !out) { set_error("rt_camera_from_lookat: null pointer"); return RT_ERR_INVALID_ARG; }
    const double theta = vfov_deg * 0.017453292519943295;   // Math.toRadians (Java 9+)
    const double h = std::tan(theta / 2.0);
    const double vh = 2.0 * h;
    const double vw = aspect * vh;
    auto unit = [](const double a[3], double r[3]) {         // Vec3.unitVector = v.multiply(1/len)
        const double len = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        const double inv = 1.0 / len;
        r[0] = a[0] * inv; r[1] = a[1] * inv; r[2] = a[2] * inv;
    };
    auto cross = [](const double a[3], const double b[3], double r[3]) {
        r[0] = a[1] * b[2] - a[2] * b[1];
        r[1] = a[2] * b[0] - a[0] * b[2];
        r[2] = a[0] * b[1] - a[1] * b[0];
    };
    double wd[3] = {origin[0] - lookat[0], origin[1] - lookat[1], origin[2] - lookat[2]};
    double w[3], c[3], u[3], v[3];
    unit(wd, w);
    cross(vup, w, c);
    unit(c, u);
    cross(w, u, v);
    double hor[3], ver[3], llc[3];
    for (int k = 0; k < 3; ++k) {
        hor[k] = u[k] * vw;
        ver[k] = v[k] * vh;
    }
    for (int k = 0; k < 3; ++k) {
        // origin.sub(horizontal.div(2.0)).sub(vertical.div(2.0)).sub(w); div(t) = multiply(1.0/t)
        llc[k] = ((origin[k] - hor[k] * (1.0 / 2.0)) - ver[k] * (1.0 / 2.0)) - w[k];
    }
    std::memset(out, 0, sizeof *out);
    for (int k = 0; k < 3; ++k) {
        out->origin[k] = (float)origin[k];
        out->lower_left[k] = (float)llc[k];
        out->horizontal[k] = (float)hor[k];
        out->vertical[k] = (float)ver[k];
    }
    out->frame_count = 0;
    out->sky_enabled = 1;
    return RT_OK;
}

// -------------------------------------------------------------------- OBJ --
//
// SceneBuilder.loadModel (SceneBuilder.java:144) reads OBJ files through
// Assimp (LWJGL-assimp 3.3.6, Assimp 5.x):
// aiImportFile(path, aiProcess_Triangulate | aiProcess_JoinIdenticalVertices),
// then keeps the 3-index faces mesh by mesh, face by face.  Restated here from
// Assimp's published sources (parity vs a real Assimp run is unpinned: the
// library is not in this image):
//  * numbers: fast_atoreal_move<float> (fast_atof.h), NOT a correctly rounded
//    strtof: the integer digits become a float, the fraction digits (at most
//    15) a double times 10^-digits, cast to float and added in float (4.9% of
//    FinalBaseMesh's coordinates differ from strtof by one ulp);
//  * 'v' lines: 3 components, 4 (x/w, y/w, z/w) or 6 (xyz + a colour);
//  * faces of 1-2 indices are points / lines (the Java loop skips them);
//  * aiProcess_Triangulate (TriangulateProcess.cpp): a quad is fanned from its
//    concave corner (angle sum > pi), else from corner 0; a larger polygon is
//    projected along its Newell normal's largest axis and ear-clipped; when no
//    ear is found twice round, the rest of the polygon is dropped (Assimp logs
//    "Failed to triangulate polygon (no ear found)" and keeps the ears so far).
// Triangles come out in file order (Assimp splits meshes at material changes
// but keeps their order of appearance).

struct rt_mesh {
    std::vector<float> v;            // xyz per vertex (as parsed, float like aiVector3D)
    std::vector<uint32_t> tri;       // 3 vertex indices per triangle
};

namespace {

// strtoul10_64 (fast_atof.h): decimal digits into a uint64; with max_digits,
// stops after that many digits and skips the rest.  No digit at all: Assimp
// throws (*bad = true here).  Overflow returns 0 and leaves the cursor where
// it was (Assimp logs a warning and carries on).
uint64_t ai_strtoul10_64(const char* in, const char** out, unsigned* max_inout, bool* bad = nullptr) {
    unsigned cur = 0;
    uint64_t value = 0;
    const char* p = in;
    if (*p < '0' || *p > '9') {
        if (bad) *bad = true;
        return 0;
    }
    while (*p >= '0' && *p <= '9') {
        const uint64_t nv = value * 10 + (uint64_t)(*p - '0');
        if (nv < value) { if (out) *out = in; return 0; }
        value = nv;
        ++p;
        ++cur;
        if (max_inout && *max_inout == cur) {
            while (*p >= '0' && *p <= '9') ++p;
            if (out) *out = p;
            return value;
        }
    }
    if (out) *out = p;
    if (max_inout) *max_inout = cur;
    return value;
}

// fast_atoreal_move<float> (fast_atof.h).  false = Assimp throws (the import
// fails and SceneBuilder skips the model).
bool ai_fast_atof(const char* c, float* out) {
    static const double kTable[16] = {0.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001,
                                      0.00000001, 0.000000001, 0.0000000001, 0.00000000001,
                                      0.000000000001, 0.0000000000001, 0.00000000000001,
                                      0.000000000000001};
    float f = 0.f;
    const bool inv = (*c == '-');
    if (inv || *c == '+') ++c;
    if ((c[0] == 'N' || c[0] == 'n') && strncasecmp(c, "nan", 3) == 0) {
        *out = std::numeric_limits<float>::quiet_NaN();
        return true;
    }
    if ((c[0] == 'I' || c[0] == 'i') && strncasecmp(c, "inf", 3) == 0) {
        *out = inv ? -std::numeric_limits<float>::infinity() : std::numeric_limits<float>::infinity();
        return true;
    }
    const bool comma = true;
    if (!(c[0] >= '0' && c[0] <= '9') && !((c[0] == '.' || (comma && c[0] == ',')) && c[1] >= '0' && c[1] <= '9'))
        return false;
    if (*c != '.' && (!comma || c[0] != ',')) f = (float)ai_strtoul10_64(c, &c, nullptr);
    if ((*c == '.' || (comma && c[0] == ',')) && c[1] >= '0' && c[1] <= '9') {
        ++c;
        unsigned diff = 15;                         // AI_FAST_ATOF_RELAVANT_DECIMALS
        double pl = (double)ai_strtoul10_64(c, &c, &diff);
        pl *= kTable[diff];
        f += (float)pl;
    } else if (*c == '.') {
        ++c;
    }
    if (*c == 'e' || *c == 'E') {
        ++c;
        const bool einv = (*c == '-');
        if (einv || *c == '+') ++c;
        bool bad = false;
        float e = (float)ai_strtoul10_64(c, &c, nullptr, &bad);
        if (bad) return false;                      // "1e": no exponent digits, Assimp throws
        if (einv) e = -e;
        f *= std::pow(10.0f, e);
    }
    if (inv) f = -f;
    *out = f;
    return true;
}

struct V3 { float x, y, z; };
struct V2 { float x, y; };

// aiVector3t::Normalize: *this /= Length(), operator/= multiplies by the
// float reciprocal and leaves a zero vector alone.
V3 ai_normalize(V3 a) {
    const float len = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    if (len == 0.f) return a;
    const float inv = 1.0f / len;
    return {a.x * inv, a.y * inv, a.z * inv};
}

// PolyTools.h
double ai_area2d(const V2& v1, const V2& v2, const V2& v3) {
    return 0.5 * (v1.x * ((double)v3.y - v2.y) + v2.x * ((double)v1.y - v3.y) + v3.x * ((double)v2.y - v1.y));
}
bool ai_on_left_side(const V2& p0, const V2& p1, const V2& p2) { return ai_area2d(p0, p2, p1) > 0; }
bool ai_point_in_triangle(const V2& p0, const V2& p1, const V2& p2, const V2& pp) {
    const V2 v0 = {p1.x - p0.x, p1.y - p0.y}, v1 = {p2.x - p0.x, p2.y - p0.y}, v2 = {pp.x - p0.x, pp.y - p0.y};
    double dot00 = v0.x * v0.x + v0.y * v0.y;       // aiVector2D dot products are float
    double dot11 = v1.x * v1.x + v1.y * v1.y;
    const double dot01 = v0.x * v1.x + v0.y * v1.y;
    const double dot02 = v0.x * v2.x + v0.y * v2.y;
    const double dot12 = v1.x * v2.x + v1.y * v2.y;
    const double denom = dot00 * dot11 - dot01 * dot01;
    if (denom == 0.0) return false;
    const double inv = 1.0 / denom;
    dot11 = (dot11 * dot02 - dot01 * dot12) * inv;
    dot00 = (dot00 * dot12 - dot01 * dot02) * inv;
    return (dot11 > 0) && (dot00 > 0) && (dot11 + dot00 < 1);
}

// TriangulateProcess::TriangulateMesh for one face of >= 3 indices: appends
// its triangles (vertex indices) to tri.
void ai_triangulate(const std::vector<float>& verts, const std::vector<uint32_t>& idx, std::vector<uint32_t>& tri) {
    auto P = [&](uint32_t i) { return V3{verts[3 * i], verts[3 * i + 1], verts[3 * i + 2]}; };
    const int max = (int)idx.size();
    if (max == 3) { tri.insert(tri.end(), idx.begin(), idx.end()); return; }
    if (max == 4) {
        // quads have at most one concave corner: fan from it
        unsigned start = 0;
        for (unsigned i = 0; i < 4; ++i) {
            const V3 v0 = P(idx[(i + 3) % 4]), v1 = P(idx[(i + 2) % 4]), v2 = P(idx[(i + 1) % 4]), v = P(idx[i]);
            const V3 left = ai_normalize({v0.x - v.x, v0.y - v.y, v0.z - v.z});
            const V3 diag = ai_normalize({v1.x - v.x, v1.y - v.y, v1.z - v.z});
            const V3 right = ai_normalize({v2.x - v.x, v2.y - v.y, v2.z - v.z});
            const float angle = std::acos(left.x * diag.x + left.y * diag.y + left.z * diag.z) +
                                std::acos(right.x * diag.x + right.y * diag.y + right.z * diag.z);
            if (angle > 3.14159265358979323846f) { start = i; break; }   // AI_MATH_PI_F
        }
        const uint32_t t[6] = {idx[start], idx[(start + 1) % 4], idx[(start + 2) % 4],
                               idx[start], idx[(start + 2) % 4], idx[(start + 3) % 4]};
        tri.insert(tri.end(), t, t + 6);
        return;
    }
    // Newell normal (NewellNormal<3,3,3>, float sums)
    float sxy = 0.f, syz = 0.f, szx = 0.f;
    for (int k = 0; k < max; ++k) {
        const V3 a = P(idx[k]), b = P(idx[(k + 1) % max]), c = P(idx[(k + 2) % max]);
        sxy += b.x * (c.y - a.y);
        syz += b.y * (c.z - a.z);
        szx += b.z * (c.x - a.x);
    }
    const float nx = syz, ny = szx, nz = sxy;
    const float ax = nx > 0 ? nx : -nx, ay = ny > 0 ? ny : -ny, az = nz > 0 ? nz : -nz;
    int ac = 0, bc = 1;                              // drop z: project to xy
    float inv = nz;
    if (ax > ay) {
        if (ax > az) { ac = 1; bc = 2; inv = nx; }   // drop x
    } else if (ay > az) {
        ac = 2; bc = 0; inv = ny;                    // drop y
    }
    if (inv < 0.f) std::swap(ac, bc);
    std::vector<V2> tv(max);
    std::vector<char> done(max, 0);
    for (int k = 0; k < max; ++k) tv[k] = {verts[3 * idx[k] + ac], verts[3 * idx[k] + bc]};
    std::vector<int> out;                            // polygon-local corners, 3 per triangle
    int num = max, ear = 0, prev = max - 1, next = 0, tmp;
    while (num > 3) {
        int found = 0;
        for (ear = next;; prev = ear, ear = next) {
            for (next = ear + 1; done[(next >= max ? next = 0 : next)]; ++next) {}
            if (next < ear && ++found == 2) break;
            const V2 &p1 = tv[ear], &p0 = tv[prev], &p2 = tv[next];
            if (ai_on_left_side(p0, p2, p1)) continue;          // must be convex
            for (tmp = 0; tmp < max; ++tmp) {                   // and hold no other corner
                const V2& q = tv[tmp];
                const bool same1 = q.x == p1.x && q.y == p1.y, same2 = q.x == p2.x && q.y == p2.y,
                           same0 = q.x == p0.x && q.y == p0.y;
                if (!same1 && !same2 && !same0 && ai_point_in_triangle(p0, p1, p2, q)) break;
            }
            if (tmp != max) continue;
            break;                                              // an ear
        }
        if (found == 2) { num = 0; break; }                     // no ear: the rest is dropped
        out.push_back(prev); out.push_back(ear); out.push_back(next);
        done[ear] = 1;
        --num;
    }
    if (num > 0) {                                              // the last three corners
        for (tmp = 0; done[tmp]; ++tmp) {}
        out.push_back(tmp);
        for (++tmp; done[tmp]; ++tmp) {}
        out.push_back(tmp);
        for (++tmp; done[tmp]; ++tmp) {}
        out.push_back(tmp);
    }
    for (int k : out) tri.push_back(idx[k]);
}

bool parse_index(const char* tok, size_t nverts, uint32_t* out) {
    char* endp = nullptr;
    long k = std::strtol(tok, &endp, 10);
    if (endp == tok) return false;
    if (k < 0) k = (long)nverts + k + 1;               // relative index
    if (k < 1 || (size_t)k > nverts) return false;
    *out = (uint32_t)(k - 1);
    return true;
}

}  // namespace

int rt_mesh_load_obj(const char* path, rt_mesh** out) {
    if (!path || !out) { set_error("rt_mesh_load_obj: null pointer"); return RT_ERR_INVALID_ARG; }
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) { set_error("rt_mesh_load_obj: cannot open %s: %s", path, std::strerror(errno)); return RT_ERR_IO; }
    rt_mesh* m = new (std::nothrow) rt_mesh;
    if (!m) { std::fclose(f); set_error("rt_mesh_load_obj: out of memory"); return RT_ERR_OOM; }
    std::vector<char> line(1 << 16);
    std::vector<uint32_t> face;
    std::vector<std::string> tok;
    size_t lineno = 0;
    int rc = RT_OK;
    auto is_ws = [](char ch) { return ch == ' ' || ch == '\t' || ch == '\r' || ch == '\n'; };
    while (std::fgets(line.data(), (int)line.size(), f)) {
        ++lineno;
        const char* s = line.data();
        while (*s == ' ' || *s == '\t') ++s;
        if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) {
            tok.clear();
            for (const char* p = s + 2; *p;) {
                while (is_ws(*p)) ++p;
                if (!*p) break;
                const char* e = p;
                while (*e && !is_ws(*e)) ++e;
                tok.emplace_back(p, e);
                p = e;
            }
            // ObjFileParser::getNumComponentsInDataDefinition: only the tokens
            // that start like a number count (ParsingUtils.h IsNumeric: a
            // digit, '-' or '+'; or nan / inf), so a trailing comment does not;
            // 3, 4 or 6 read that many words in order (getVector3 /
            // getHomogeneousVector3 / getTwoVectors3, the colour parsed and
            // dropped); any other count adds no vertex at all.
            size_t n = 0;
            for (const std::string& t : tok) {
                const char* q = t.c_str();
                if ((*q >= '0' && *q <= '9') || *q == '-' || *q == '+' || strncasecmp(q, "nan", 3) == 0 ||
                    strncasecmp(q, "inf", 3) == 0)
                    ++n;
            }
            if (n != 3 && n != 4 && n != 6) continue;
            float c[6] = {0.f, 0.f, 0.f, 1.f, 0.f, 0.f};
            bool ok = true;
            for (size_t k = 0; ok && k < n; ++k) ok = ai_fast_atof(tok[k].c_str(), &c[k]);
            if (ok && n == 4) {
                if (c[3] == 0.f) ok = false;                    // Assimp: division by zero
                else { c[0] /= c[3]; c[1] /= c[3]; c[2] /= c[3]; }
            }
            if (!ok) { rc = RT_ERR_IO; set_error("rt_mesh_load_obj: %s:%zu: bad vertex", path, lineno); break; }
            m->v.insert(m->v.end(), c, c + 3);
        } else if (s[0] == 'f' && (s[1] == ' ' || s[1] == '\t')) {
            face.clear();
            const char* p = s + 2;
            const size_t nv = m->v.size() / 3;
            while (*p) {
                while (is_ws(*p)) ++p;
                if (!*p) break;
                uint32_t idx;
                if (!parse_index(p, nv, &idx)) { rc = RT_ERR_IO; break; }
                face.push_back(idx);
                while (*p && !is_ws(*p)) ++p;
            }
            if (rc) { set_error("rt_mesh_load_obj: %s:%zu: bad face", path, lineno); break; }
            if (face.size() < 3) continue;                 // points / lines are not triangles
            ai_triangulate(m->v, face, m->tri);
        }
    }
    std::fclose(f);
    if (rc) { delete m; return rc; }
    *out = m;
    return RT_OK;
}

size_t rt_mesh_tri_count(const rt_mesh* mesh) { return mesh ? mesh->tri.size() / 3 : 0; }

int rt_mesh_transform(const rt_mesh* mesh, const double scale[3], const double position[3],
                      double* out) {
    if (!mesh || !scale || !position || !out) { set_error("rt_mesh_transform: null pointer"); return RT_ERR_INVALID_ARG; }
    const size_t nt = mesh->tri.size() / 3;
    for (size_t t = 0; t < nt; ++t) {
        for (int c = 0; c < 3; ++c) {
            const float* v = &mesh->v[3 * mesh->tri[3 * t + c]];
            for (int k = 0; k < 3; ++k)   // v.multiply(scale).add(position), SceneBuilder.java:172
                out[t * 9 + c * 3 + k] = (double)v[k] * scale[k] + position[k];
        }
    }
    return RT_OK;
}

int rt_mesh_free(rt_mesh* mesh) {
    delete mesh;
    return RT_OK;
}

// ------------------------------------------------------------- procedural --

int rt_mesh_procedural(size_t n_tris, uint64_t seed, const double bmin[3], const double bmax[3],
                       double* out) {
    if (!bmin || !bmax || !out) { set_error("rt_mesh_procedural: null pointer"); return RT_ERR_INVALID_ARG; }
    if (n_tris < 8 || (n_tris & 1)) { set_error("rt_mesh_procedural: n_tris must be even and >= 8"); return RT_ERR_INVALID_ARG; }
    // Lat-long shell: nu columns, nr latitude bands (2 pole fans + nr-2 quad
    // bands) gives 2*nu*(nr-1) triangles; nu = the divisor of n/2 closest to
    // sqrt(n) (so the facets are roughly square).
    const size_t m = n_tris / 2;
    size_t nu = 0;
    const double target = std::sqrt((double)n_tris);
    for (size_t d = 1; d * d <= m; ++d) {
        if (m % d) continue;
        for (size_t c : {d, m / d})
            if (c >= 3 && (nu == 0 || std::fabs((double)c - target) < std::fabs((double)nu - target))) nu = c;
    }
    if (nu == 0) nu = m;
    const size_t nr = m / nu + 1;
    // Seeded radial displacement: a sum of 6 low-frequency products of sines.
    double amp[6], fu[6], fv[6], pu[6], pv[6];
    uint64_t s = seed;
    auto uni = [&s]() { s = splitmix64(s); return (double)(s >> 11) * (1.0 / 9007199254740992.0); };
    for (int k = 0; k < 6; ++k) {
        amp[k] = 0.02 + 0.02 * uni();
        fu[k] = (double)(1 + (int)(uni() * 7));
        fv[k] = (double)(1 + (int)(uni() * 7));
        pu[k] = 6.283185307179586 * uni();
        pv[k] = 6.283185307179586 * uni();
    }
    const double c[3] = {(bmin[0] + bmax[0]) / 2, (bmin[1] + bmax[1]) / 2, (bmin[2] + bmax[2]) / 2};
    const double r[3] = {(bmax[0] - bmin[0]) / 2, (bmax[1] - bmin[1]) / 2, (bmax[2] - bmin[2]) / 2};
    auto point = [&](size_t i, size_t j, double p[3]) {   // i = ring 0..nr, j = column
        const double th = 3.141592653589793 * (double)i / (double)nr;
        const double ph = 6.283185307179586 * (double)(j % nu) / (double)nu;
        double disp = 0.0;
        for (int k = 0; k < 6; ++k) disp += amp[k] * std::sin(fu[k] * ph + pu[k]) * std::sin(fv[k] * th + pv[k]);
        const double rad = 0.86 + disp;                     // in [0.74, 0.98] of the half extents
        p[0] = c[0] + r[0] * rad * std::sin(th) * std::cos(ph);
        p[1] = c[1] + r[1] * rad * std::cos(th);
        p[2] = c[2] + r[2] * rad * std::sin(th) * std::sin(ph);
    };
    size_t t = 0;
    auto emit = [&](const double* a, const double* b, const double* cc) {
        std::memcpy(out + 9 * t, a, 24);
        std::memcpy(out + 9 * t + 3, b, 24);
        std::memcpy(out + 9 * t + 6, cc, 24);
        ++t;
    };
    double top[3], bot[3];
    point(0, 0, top);
    point(nr, 0, bot);
    for (size_t j = 0; j < nu; ++j) {
        double a[3], b[3];
        point(1, j, a);
        point(1, j + 1, b);
        emit(top, b, a);
    }
    for (size_t i = 1; i + 1 < nr; ++i) {
        for (size_t j = 0; j < nu; ++j) {
            double p00[3], p01[3], p10[3], p11[3];
            point(i, j, p00);
            point(i, j + 1, p01);
            point(i + 1, j, p10);
            point(i + 1, j + 1, p11);
            emit(p00, p01, p11);
            emit(p00, p11, p10);
        }
    }
    for (size_t j = 0; j < nu; ++j) {
        double a[3], b[3];
        point(nr - 1, j, a);
        point(nr - 1, j + 1, b);
        emit(bot, a, b);
    }
    if (t != n_tris) { set_error("rt_mesh_procedural: internal count mismatch %zu != %zu", t, n_tris); return RT_ERR_INVALID_ARG; }
    return RT_OK;
}

}  // extern "C"
