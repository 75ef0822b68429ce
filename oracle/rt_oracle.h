/*
 * rt_oracle.h — CPU oracle of the path-trace path.  TEST INFRASTRUCTURE ONLY
 * (see rt_oracle.c for the rules of use and the parity status).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

typedef struct {                      /* the 80-B CameraUBO (VulkanEngine.java:387-395) */
    float origin[4], lower_left[4], horizontal[4], vertical[4];
    int32_t frame_count, sky_enabled, pad[2];
} orc_camera;

typedef struct {
    uint64_t pixels, segments, node_visits, tri_tests, mat_reads;
} orc_counts;

uint32_t orc_pcg(uint32_t v);
float    orc_random_float(uint32_t* seed);
void     orc_random_in_unit_sphere(uint32_t* seed, float out[3]);
int      orc_hit_aabb(const float origin[3], const float dir[3], const float bmin[3],
                      const float bmax[3], float t_min, float t_max);
int      orc_hit_triangle(const float origin[3], const float dir[3], const float v0[3],
                          const float v1[3], const float v2[3], float* closest_t, float normal[3]);
int      orc_hit_sphere(const float origin[3], const float dir[3], const float centre_radius[4],
                        float* closest_t, float normal[3]);   /* extension ORC_EXT_SPHERES */
int      orc_scatter(const float material[4], uint32_t* seed, const float dir_in[3],
                     const float hit_pos[3], const float normal[3], float att[3], float dir_out[3]);

/* Renders rows y0, y0+row_step, ... of the tile [x0,x0+tile_w) x [y0,y0+tile_h)
 * of a width x height frame.  Output rows are packed (row r of the output =
 * frame row y0 + r*row_step).  n_threads: 0 = OpenMP default. */
int orc_render(const void* vertices, size_t vertex_bytes,
               const void* materials, size_t material_bytes,
               const void* bvh_nodes, size_t bvh_bytes,
               const orc_camera* cam, int width, int height, int max_bounces,
               int x0, int y0, int tile_w, int tile_h, int row_step,
               uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads);
/* Same, plus profile[pixel * max_bounces + b] = node visits (low 20 bits) |
 * triangle tests << 20 of bounce b (0 where the path ended earlier).
 * An analysis aid for kernel design (tools/simd_model.py). */
int orc_render_profile(const void* vertices, size_t vertex_bytes,
                       const void* materials, size_t material_bytes,
                       const void* bvh_nodes, size_t bvh_bytes,
                       const orc_camera* cam, int width, int height, int max_bounces,
                       int x0, int y0, int tile_w, int tile_h, int row_step,
                       uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads,
                       uint32_t* profile);
/* Non-reference extensions, the semantics the GPU path's
 * option "extensions" implements; bit-exact against it, unpinned against any
 * reference (the reference has none of them):
 *   ORC_EXT_SKY_TOGGLE  a miss is black when cam->sky_enabled == 0
 *   ORC_EXT_EMISSIVE    a type-3 hit ends the path with attenuation * albedo
 *   ORC_EXT_ACCUMULATE  seed += frame_count * W * H; accum (3 floats per output
 *                       pixel, packed like out_rgba) holds the running sum of the
 *                       linear colour (frame_count 0 overwrites it); the output is
 *                       sqrt(sum / (frame_count + 1))
 *   ORC_EXT_SPHERES     orc_render_spheres' spheres (8 floats each: centre.xyz,
 *                       radius, albedo.rgb, material type) are tested after the
 *                       BVH walk of every segment, in index order, against
 *                       (T_MIN, closest_t): oc = o - c, a = dot(d,d), half_b =
 *                       dot(oc,d), disc = half_b^2 - a*(dot(oc,oc) - r*r); the
 *                       root (-half_b - sqrt(disc))/a, else (-half_b +
 *                       sqrt(disc))/a; normal (p - c)/r turned to face the ray.
 *                       A sphere hit shades with the sphere's material and
 *                       counts one material read; node / triangle counts are
 *                       unchanged. */
#define ORC_EXT_SKY_TOGGLE 1
#define ORC_EXT_EMISSIVE   2
#define ORC_EXT_ACCUMULATE 4
#define ORC_EXT_SPHERES    8
int orc_render_ext(const void* vertices, size_t vertex_bytes,
                   const void* materials, size_t material_bytes,
                   const void* bvh_nodes, size_t bvh_bytes,
                   const orc_camera* cam, int width, int height, int max_bounces,
                   int x0, int y0, int tile_w, int tile_h, int row_step,
                   uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads,
                   int ext, float* accum);
int orc_render_spheres(const void* vertices, size_t vertex_bytes,
                       const void* materials, size_t material_bytes,
                       const void* bvh_nodes, size_t bvh_bytes,
                       const orc_camera* cam, int width, int height, int max_bounces,
                       int x0, int y0, int tile_w, int tile_h, int row_step,
                       uint8_t* out_rgba, float* out_radiance, orc_counts* counts, int n_threads,
                       int ext, float* accum, const float* spheres, int n_spheres);
#endif
