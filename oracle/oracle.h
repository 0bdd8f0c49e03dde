/*
 * oracle.h — CPU parity oracle for the MI355X path tracer.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (raytracinginoneweekendinrust_amd/)
 * links, loads or calls this; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg do, and only as the checker / reported CPU baseline.
 *
 * What it is: a plain-C restatement of the reference's per-pixel hot path
 * (jalberse/RayTracingInOneWeekendInRust, crate `shimmer`), following its
 * trait-object structure literally: recursive `ray_color`, ordered
 * `HittableList::hit`, recursive `BvhNode::hit` with the reference's quirks,
 * per-candidate `HitRecord` construction, and the reference's random-draw
 * order. Every function cites the file:line it follows.
 *
 * Parity status:
 *  - The reference itself cannot be compiled here (Rust; no cargo/rustc) and its
 *    RNG is OS-seeded `thread_rng`, so no bit-level golden output of the
 *    reference exists. The oracle is pinned by the reference's own unit tests and
 *    doc-comment known answers (src/aabb.rs:73-140, src/renderer.rs:311-377,
 *    src/geometry/sphere.rs:37-40), by Random123's published Philox KATs, and by
 *    numeric-spec checks against Python's libm. Radiance output is therefore
 *    "parity pinned by component KATs", not by reference renders.
 *  - Random streams: rand 0.8.5 ChaCha12 `thread_rng` is replaced by
 *    Philox4x32-10 keyed (seed, pixel, sample); the f32 constructions of
 *    `Standard` and `gen_range` are restated exactly.
 *  - Transcendentals: libm (what Rust's f32 methods call) is replaced by
 *    include/rt_numeric_spec.h unless ORACLE_FLAG_LIBM is set.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#include "../include/rt.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_FLAG_RECURSIVE 1u /* literal src/ray.rs:51-55 recursion e + a*(...)   */
#define ORACLE_FLAG_LIBM 2u      /* use libm sinf/acosf/atan2f/logf/tanf/cosf        */

typedef struct oracle_options {
    uint32_t flags;
    uint32_t num_threads; /* 0 = all online cores */
} oracle_options;

typedef struct oracle_counters {
    uint64_t samples;       /* camera samples                                  */
    uint64_t segments;      /* ray_color calls that intersected the world      */
    uint64_t hits;          /* segments whose world hit produced a HitRecord   */
    uint64_t node_visits;   /* BvhNode::hit calls (AABB tests)                 */
    uint64_t sphere_tests;  /* Sphere::hit calls                               */
    uint64_t msphere_tests; /* MovingSphere::hit calls                         */
    uint64_t rect_tests;    /* Xy/Xz/YzRect::hit calls (cube faces included)   */
    uint64_t tri_tests;     /* Tri::hit calls                                  */
    uint64_t medium_tests;  /* ConstantMedium::hit calls                       */
    uint64_t texel_fetches; /* ImageTexture::value calls                       */
    double seconds;         /* wall time of the render loop                    */
    uint32_t threads;       /* worker threads used                             */
} oracle_counters;

/* Renders the pixels of the shard selected by params (8x8 blocks b with
 * b % shard_count == shard_index) into out (W*H*3, row 0 = reference y = 0). */
int oracle_render(const rt_scene_desc* scene, const rt_camera_desc* camera,
                  const rt_render_params* params, const oracle_options* options,
                  float* out, oracle_counters* counters);

/* oracle_render for a constructed Camera (src/camera.rs:6-27), as Renderer::render
 * receives it. */
int oracle_render_camera(const rt_scene_desc* scene, const rt_camera* camera,
                         const rt_render_params* params, const oracle_options* options,
                         float* out, oracle_counters* counters);

/* Radiance of one camera sample (forward or recursive per flags). */
int oracle_sample(const rt_scene_desc* scene, const rt_camera_desc* camera,
                  const rt_render_params* params, uint32_t flags, uint32_t x,
                  uint32_t y, uint32_t sample, float rgb[3]);

const char* oracle_last_error(void);

/* Component restatements exposed for known-answer tests. */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t oracle_tile(uint32_t w, uint32_t h, uint32_t tw, uint32_t th, rt_tile* out,
                     uint32_t cap);                                  /* renderer.rs:242 */
int oracle_aabb_hit(const float mn[3], const float mx[3], const float o[3],
                    const float d[3], float tmin, float tmax);       /* aabb.rs:28   */
int oracle_aabb_union(const float* a /*6 or NULL*/, const float* b /*6 or NULL*/,
                      float out[6]);                                 /* aabb.rs:43   */
void oracle_sphere_uv(const float p[3], float uv[2]);                /* sphere.rs:41 */
/* Camera::new basis: origin, horizontal, vertical, lower_left, u, v (18 floats),
 * lens_radius, time_low, time_scale. */
void oracle_camera_basis(const rt_camera_desc* cam, float out[21]);
/* Perlin Turbulence value of a Marble seed at p (noise 0.8.2 restatement). */
double oracle_turbulence(uint32_t seed, const double p[3]);
/* Leaf order of Bvh::new over n items with box_compare keys keys[3 i + axis] (bvh.rs:249-333). */
int oracle_bvh_order(const float* keys, uint32_t n, uint64_t seed, uint32_t* order);
/* Host numeric spec evaluation (ops of rt_device_numeric_eval; 8 = rt_cosf, 9 = rt_tanf). */
void oracle_numeric_eval(int op, const double* a, const double* b, double* out, uint32_t n);

#ifdef __cplusplus
}
#endif

#endif
