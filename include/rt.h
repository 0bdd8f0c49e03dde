/*
 * rt.h — C ABI of the MI355X (gfx950) path-tracing hot path.
 *
 * Drop-in boundary for jalberse/RayTracingInOneWeekendInRust (crate `shimmer`):
 * everything below `Renderer::render` (src/renderer.rs:42-105) — the per-pixel
 * sample loop `Renderer::get_color` (src/renderer.rs:129-149), `Camera::get_ray`
 * (src/camera.rs:96-106), `Ray::ray_color` (src/ray.rs:32-62), `Hittable::hit`
 * for every geometry / acceleration type (src/hittable.rs, src/bvh.rs,
 * src/aabb.rs, src/geometry/), `Material::scatter/emit` (src/materials/) and
 * `Texture::value` (src/textures/) — runs as one HIP kernel launch per frame.
 *
 * The Rust side keeps its trait surface. Its scene (an `Arc<dyn Hittable>`
 * graph) is lowered to the flat node IR below: one `rt_node` per reference
 * constructor call (`Sphere::new`, `Bvh::new`, `RotateY::new`, ...), children
 * referenced by node index. Shared `Arc`s are shared indices. INTEGRATION.md
 * shows the `extern "C"` block the reference would add.
 *
 * Conventions
 *  - Every entry point returns RT_OK (0) or a negative rt_status. On failure
 *    rt_last_error() returns a per-thread message. No entry point aborts.
 *  - Caller keeps ownership of every pointer it passes in; the library copies.
 *  - Images are linear RGB f32, W*H*3, row 0 = the reference's y = 0 (the
 *    bottom row; src/renderer.rs:141-142, written top-down by write_ppm).
 */
#ifndef RT_H
#define RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 2

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID = -1,     /* bad argument / malformed scene IR               */
    RT_ERR_UNSUPPORTED = -2, /* IR shape the device path does not lower         */
    RT_ERR_HIP = -3,         /* HIP runtime error (message has hipGetErrorString) */
    RT_ERR_OOM = -4,         /* host or device allocation failed                */
    RT_ERR_NO_DEVICE = -5,   /* no gfx950 device visible                        */
    RT_ERR_IO = -6           /* asset file missing / unreadable                 */
} rt_status;

/* ------------------------------------------------------------------------ */
/* Scene IR: one node per reference constructor call.                        */
/* ------------------------------------------------------------------------ */
typedef enum rt_node_kind {
    /* textures — trait Texture, src/textures/texture.rs:3-5 */
    RT_TEX_SOLID = 1,         /* f[0..3] color                      solid_color.rs:10   */
    RT_TEX_CHECKER = 2,       /* f[0] scale, ref[0] even, ref[1] odd checker.rs:14      */
    RT_TEX_MARBLE = 3,        /* f[0] scale, seed = Perlin seed      marble.rs:13        */
    RT_TEX_IMAGE = 4,         /* ref[0] width, ref[1] height, seed = byte offset of the
                                 RGB8 texels in rt_scene_desc.image_data  image_texture.rs:13 */
    /* materials — trait Material, src/materials/material.rs:16-23 */
    RT_MAT_LAMBERTIAN = 16,   /* ref[0] albedo texture               lambertian.rs:23    */
    RT_MAT_METAL = 17,        /* f[0..3] albedo, f[3] fuzz (raw; clamped like metal.rs:20) */
    RT_MAT_DIELECTRIC = 18,   /* f[0] index of refraction            dialectric.rs:19    */
    RT_MAT_DIFFUSE_LIGHT = 19,/* ref[0] emission texture             diffuse_light.rs:14 */
    RT_MAT_ISOTROPIC = 20,    /* ref[0] albedo texture               isotropic.rs:20     */
    /* hittables — trait Hittable, src/hittable.rs:64-82 */
    RT_OBJ_SPHERE = 32,       /* f[0..3] center, f[3] radius, ref[0] material  sphere.rs:26 */
    RT_OBJ_MOVING_SPHERE = 33,/* f[0..3] c0, f[3..6] c1, f[6] t0, f[7] t1, f[8] radius,
                                 ref[0] material                     moving_sphere.rs:29 */
    RT_OBJ_XY_RECT = 34,      /* f = x0,x1,y0,y1,z ; ref[0] material rectangle.rs:24     */
    RT_OBJ_XZ_RECT = 35,      /* f = x0,x1,z0,z1,y ; ref[0] material rectangle.rs:86     */
    RT_OBJ_YZ_RECT = 36,      /* f = y0,y1,z0,z1,x ; ref[0] material rectangle.rs:148    */
    RT_OBJ_CUBE = 37,         /* f[0..3] min, f[3..6] max, ref[0] material  cube.rs:23   */
    RT_OBJ_TRI = 38,          /* f[0..9] p0,p1,p2, ref[0] material   triangle.rs:21      */
    RT_OBJ_LIST = 39,         /* ref[0] first index into list_items, ref[1] count
                                                                     hittable.rs:84-98   */
    RT_OBJ_BVH = 40,          /* ref[0] LIST node, f[0] time0, f[1] time1,
                                 seed = split-axis stream seed        bvh.rs:46-62
                                 ref[1] = 1: Bvh::with_predictor (an HRPP table,
                                 used only under RT_FLAG_HRPP)        bvh.rs:69-80        */
    RT_OBJ_TRANSLATE = 41,    /* ref[0] child, f[0..3] displacement  instance.rs:23      */
    RT_OBJ_ROTATE_Y = 42,     /* ref[0] child, f[0] degrees          instance.rs:63      */
    RT_OBJ_CONSTANT_MEDIUM = 43,/* ref[0] boundary, ref[1] phase albedo texture,
                                 f[0] density                        hittable.rs:150-174 */
    RT_OBJ_BVH_TREE = 44      /* an already built Bvh (bvh.rs:38-43): its BvhNode array
                                 as the reference holds it. ref[0] first rt_bvh_node of
                                 the tree in rt_scene_desc.bvh_nodes, ref[1] node count,
                                 ref[2] root_index (relative to ref[0]), f[0] / f[1]
                                 ignored (the reference's Bvh stores no shutter times),
                                 f[2] = 1: built
                                 with Bvh::with_predictor (HRPP only). Its boxes and
                                 leaf nodes decide the visit set and every DFS-rank
                                 tie, as BvhNode::hit walks the array (the fast kernel
                                 may rebuild the interior levels: RT_OPT_BVH_SHAPE). */
} rt_node_kind;

/* One reference BvhNode (src/bvh.rs:228-235), children as the enum Child
 * (bvh.rs:30-33). A node's children are both Child::Hittable (the 1-2 object
 * leaves new_helper makes; a 1-object node repeats its object, bvh.rs:261-264)
 * or both Child::Index. */
#define RT_BVH_LEFT_HITTABLE 1u   /* left is Child::Hittable(IR node index)       */
#define RT_BVH_RIGHT_HITTABLE 2u  /* right is Child::Hittable(IR node index)      */
typedef struct rt_bvh_node {
    int32_t left, right;   /* Child::Index(i): node i of the same tree (relative
                              to the tree's first node); Child::Hittable: the IR
                              node index of the object (a primitive / Cube)     */
    uint32_t flags;        /* RT_BVH_*_HITTABLE                                 */
    int32_t parent;        /* Option<usize> parent, -1 = None (not needed by the
                              exact traversal; kept so the array mirrors BvhNode) */
    float bbox_min[3];     /* bounding_box: tested as given, like bvh.rs:370    */
    float bbox_max[3];
} rt_bvh_node;             /* 40 bytes */

typedef struct rt_node {
    uint32_t kind;   /* rt_node_kind */
    int32_t ref[3];  /* node indices (or counts, see kind); -1 = unused */
    float f[12];     /* numeric constructor arguments */
    uint64_t seed;   /* Perlin seed / BVH axis-stream seed / image byte offset */
} rt_node;           /* 72 bytes, no padding */

typedef struct rt_scene_desc {
    const rt_node* nodes;
    uint32_t num_nodes;
    int32_t world;              /* index of the LIST node passed as `world` */
    const int32_t* list_items;  /* children of LIST nodes, node indices */
    uint32_t num_list_items;
    uint32_t reserved0;
    const uint8_t* image_data;  /* RGB8 texels of every RT_TEX_IMAGE */
    uint64_t image_bytes;
    const rt_bvh_node* bvh_nodes; /* node arrays of every RT_OBJ_BVH_TREE (may be NULL) */
    uint32_t num_bvh_nodes;
    uint32_t reserved1;
} rt_scene_desc;

/* Raw arguments of Camera::new (src/camera.rs:44-81); the basis is derived
 * on the host exactly as the reference does (rt_camera_new). */
typedef struct rt_camera_desc {
    float look_from[3];
    float look_at[3];
    float view_up[3];
    float vfov_deg;
    float aspect_ratio;
    float aperture;
    float focus_dist;
    float time0;
    float time1;
} rt_camera_desc;

/* A constructed Camera: exactly the nine fields the reference's Camera stores
 * (src/camera.rs:6-27), which is all Renderer::render receives
 * (src/renderer.rs:42-52). Camera::get_ray (camera.rs:96-106) reads nothing else. */
typedef struct rt_camera {
    float origin[3];
    float horizontal[3];
    float vertical[3];
    float lower_left_corner[3];
    float u[3];
    float v[3];
    float lens_radius;
    float time_start;
    float time_end;
} rt_camera;

#define RT_FLAG_EXACT_BVH 1u  /* box tests use the BVH entry t_max like bvh.rs:363-417
                                 (no closest-hit pruning); results are identical
                                 except for measure-zero ties, it is slower      */
#define RT_FLAG_HRPP 2u       /* EXPERIMENT, approximate: hash-based ray path
                                 prediction on every Bvh::with_predictor BVH
                                 (src/hrpp.rs, src/bvh.rs:114-211), traversal
                                 otherwise as RT_FLAG_EXACT_BVH. Tables start
                                 empty at each launch and are filled concurrently,
                                 so results are NOT deterministic (neither are
                                 the reference's, bvh.rs:146-149)             */
/* Progressive (time-sliced) rendering: a frame of S spp rendered as slices
 * [b, e) — sample_base = b, samples_per_pixel = e - b, spp_total = S — gives the
 * one-shot image bit for bit, because every pixel's sum keeps sample order: */
#define RT_FLAG_ACCUMULATE 4u /* the slice continues the running sum already in
                                 the output instead of starting from zero      */
#define RT_FLAG_RAW_SUM 8u    /* leave the running sum in the output (no final
                                 division): every slice but the last           */
#define RT_FLAG_FRAMES_IN_FLIGHT 16u /* the caller overlaps this launch with launches on
                                 other scene handles of the same device: the
                                 streaming replay pass, whose waves would start
                                 in the other launch's drain and leave at once,
                                 is not launched; the serialized pass re-traces
                                 every handed-over sample (same bits)          */

typedef struct rt_render_params {
    uint32_t width, height;      /* image size (Renderer::from_aspect_ratio)        */
    uint32_t samples_per_pixel;  /* spp, src/renderer.rs:140                        */
    uint32_t max_depth;          /* ray_color depth, src/ray.rs:39-41               */
    uint32_t tile_width, tile_height; /* Tile::tile decomposition (must be >= 1)    */
    uint64_t seed;               /* Philox key of the per-sample random streams     */
    uint32_t sample_base;        /* global index of this call's first sample        */
    uint32_t shard_index;        /* this call renders the 8x8 pixel blocks b with   */
    uint32_t shard_count;        /*   b % shard_count == shard_index (0/1 = all)    */
    uint32_t flags;              /* RT_FLAG_*                                       */
    float background[3];         /* src/main.rs:155-164                             */
    uint32_t spp_total;          /* divisor of the final average; 0 = samples_per_pixel
                                    (set to the frame's spp for the last slice)    */
} rt_render_params;

typedef struct rt_stats {
    uint64_t segments;    /* ray segments traced (world intersections)            */
    uint64_t samples;     /* camera samples taken                                 */
    double kernel_ms;     /* device time of the render launch (rt_render only)    */
} rt_stats;

typedef struct rt_tile {
    uint32_t width, height, x_start, y_start;
} rt_tile;

/* The layouts a foreign binding mirrors byte for byte (INTEGRATION.md's #[repr(C)] structs,
 * the ctypes mirror in raytracinginoneweekendinrust_amd/_capi.py): every C or C++ compile of
 * this header checks them. */
#ifdef __cplusplus
#define RT_LAYOUT_ASSERT(cond, what) static_assert(cond, what)
#else
#define RT_LAYOUT_ASSERT(cond, what) _Static_assert(cond, what)
#endif
RT_LAYOUT_ASSERT(sizeof(rt_node) == 72 && offsetof(rt_node, ref) == 4 && offsetof(rt_node, f) == 16 &&
                     offsetof(rt_node, seed) == 64, "rt_node layout");
RT_LAYOUT_ASSERT(sizeof(rt_bvh_node) == 40 && offsetof(rt_bvh_node, bbox_min) == 16 &&
                     offsetof(rt_bvh_node, bbox_max) == 28, "rt_bvh_node layout");
RT_LAYOUT_ASSERT(sizeof(rt_scene_desc) == 64 && offsetof(rt_scene_desc, list_items) == 16 &&
                     offsetof(rt_scene_desc, image_data) == 32 && offsetof(rt_scene_desc, image_bytes) == 40 &&
                     offsetof(rt_scene_desc, bvh_nodes) == 48 && offsetof(rt_scene_desc, num_bvh_nodes) == 56,
                 "rt_scene_desc layout");
RT_LAYOUT_ASSERT(sizeof(rt_camera) == 84 && offsetof(rt_camera, lens_radius) == 72 &&
                     offsetof(rt_camera, time_end) == 80, "rt_camera layout");
RT_LAYOUT_ASSERT(sizeof(rt_render_params) == 64 && offsetof(rt_render_params, seed) == 24 &&
                     offsetof(rt_render_params, sample_base) == 32 && offsetof(rt_render_params, flags) == 44 &&
                     offsetof(rt_render_params, background) == 48 && offsetof(rt_render_params, spp_total) == 60,
                 "rt_render_params layout");
RT_LAYOUT_ASSERT(sizeof(rt_stats) == 24 && offsetof(rt_stats, kernel_ms) == 16, "rt_stats layout");

typedef struct rt_scene* rt_scene_handle;

/* ------------------------------------------------------------------------ */
/* Entry points                                                              */
/* ------------------------------------------------------------------------ */
int rt_abi_version(void);
const char* rt_last_error(void);
int rt_device_count(int* count);

/* Tile::tile, src/renderer.rs:242-296. Writes min(cap, n) tiles, returns n in *count. */
int rt_tile_image(uint32_t image_width, uint32_t image_height, uint32_t tile_width,
                  uint32_t tile_height, rt_tile* out, uint32_t cap, uint32_t* count);

/* Lower the IR to device SoA buffers on `device` (one copy in HBM). */
int rt_scene_upload(const rt_scene_desc* scene, int device, rt_scene_handle* out);
int rt_scene_free(rt_scene_handle scene);
/* counts: [entries, spheres, moving spheres, rects, tris, bvh nodes, materials,
 *          textures, max bvh depth, device bytes] */
int rt_scene_info(rt_scene_handle scene, uint64_t counts[10]);

/* Asynchronous render on `stream` (hipStream_t, NULL = default stream) into a
 * DEVICE buffer of W*H*3 floats; only the shard's pixels are written.
 * d_segments (device uint64, may be NULL) is incremented by the segments traced.
 * Renders on one scene handle are serialised: a launch waits (on the device,
 * hipStreamWaitEvent) for the previous launch on the same handle to finish,
 * whatever stream either was issued on, because they share the handle's sample
 * buffer and counters; concurrent calls from several threads are safe.
 * Memory: the handle keeps a device sample buffer (12 B per pixel and sample of a
 * chunk) sized for the largest launch it has run, at most 40% of the HBM free when it
 * grew (at least 8 GiB; rt_set_option(RT_OPT_SAMPLE_BUFFER_MB) caps it), until
 * rt_scene_free. Several handles on one device each keep their own: cap the buffer
 * when many handles share a GPU, or a later one may fall back to more chunks. */
int rt_render_launch(rt_scene_handle scene, const rt_camera_desc* camera,
                     const rt_render_params* params, float* d_out,
                     unsigned long long* d_segments, void* stream);

/* One frame over several devices of this process: scenes[i]
 * (uploaded on its own device; two handles may share a device) renders the 8x8
 * blocks b with b % n == i, all devices concurrently, and the shards are gathered
 * into host_out (W*H*3 floats, every pixel written). params->shard_count must be
 * 0 or 1. stats: segments summed, kernel_ms of the slowest device. The result is
 * bit-identical to rt_render on one device. */
int rt_render_multi(rt_scene_handle* scenes, uint32_t n, const rt_camera_desc* camera,
                    const rt_render_params* params, float* host_out, rt_stats* stats);

/* Output step of Renderer::render (src/renderer.rs:107-127) on the device.
 * rt_quantize_srgb8: palette 0.6.1 Srgb<f32> -> Srgb<u8> (clamp to [0, 1] with
 * NaN -> 0, x 255, round half away from zero; no gamma, src/utils.rs:19-23) of a
 * device image (W*H*3 floats, row 0 = bottom) into d_u8 (W*H*3 bytes, rows top to
 * bottom, as the PPM writes them); asynchronous on `stream`.
 * rt_format_ppm: the P3 body the reference prints, "r g b\n" per pixel, rows top
 * to bottom, into device buffer d_text (capacity >= 12 bytes per pixel); the
 * "P3\nW H\n255\n" header is not included. Synchronises `stream` and stores the
 * body length in *text_bytes. */
int rt_quantize_srgb8(const float* d_rgb, uint8_t* d_u8, uint32_t width, uint32_t height, void* stream);
int rt_format_ppm(const float* d_rgb, uint32_t width, uint32_t height, char* d_text, uint64_t capacity,
                  uint64_t* text_bytes, void* stream);

/* Bvh::new's leaf order (src/bvh.rs:249-333) built on the device. d_keys holds
 * n x 3 floats, item i's bounding_box(0, 0).min (the box_compare key, :420-440);
 * seed is the BVH's split-axis seed (rt_node.seed of its RT_OBJ_BVH node). Writes
 * to d_order the item indices in the order the reference recursion leaves them
 * (random axis per node, stable total_cmp sort, split at n / 2, two-item nodes
 * ordered by one comparison). Synchronises `stream`. rt_scene_upload uses it for
 * BVHs of >= 16384 items (RT_OPT_BVH_BUILD overrides: "device always" builds every
 * BVH on the device, "host always" none); the lowered tree is identical either way.
 * n < 2^31; RT_ERR_UNSUPPORTED beyond about 1.4e9 items (the split-axis draws would
 * exceed 2^32 words). Device memory: about 33 B per item for the call's duration. */
int rt_bvh_build_order(const float* d_keys, uint32_t n, uint64_t seed, uint32_t* d_order, void* stream);

/* Diagnostic options (tests, A/B runs, experiments). The library reads no environment
 * variables: each switch below is process-wide, starts at its default, and changes only
 * through rt_set_option. None is needed for production renders.
 *   RT_OPT_TUNE             traversal mode bits (kernel.hip kMode*; default 0). Bit 16 sends
 *                           the replay pass through the literal reference kernel. The product
 *                           library accepts only bits that leave the image bits unchanged
 *                           (kernel.hip kTuneExact: 1, 5, 6, 7, 16, 17, 21, 22, 24-27); any
 *                           other bit (the inexact prune-all experiment, audit and ablation
 *                           switches) is RT_ERR_INVALID there and honoured only by the
 *                           diagnostic builds (librtamd_audit.so, librtamd_ablate.so).
 *   RT_OPT_GROUP            samples per batch (1..64; 0 = automatic, the default)
 *   RT_OPT_STACK_LDS        cap on the LDS part of the traversal stack, read at upload
 *                           (>= 1; 0 = the default 19 entries); deeper stacks spill to HBM
 *   RT_OPT_SAMPLE_BUFFER_MB sample-buffer budget in MiB (0 = 40% of free HBM, the default)
 *   RT_OPT_HRPP_SLOT_BITS   log2 HRPP table slots per predictor (-1 = 22, the default; 0..28)
 *   RT_OPT_LAUNCH_LOG       1 = print the launched kernel instance and replay counts on stderr
 *   RT_OPT_BVH_BUILD        leaf ordering of BVHs at upload: 0 = device for >= 16384 items
 *                           (default), 1 = host always, 2 = device always
 *   RT_OPT_GUIDE            guided batch divisor K: a batch is at most (units left) /
 *                           (K x waves) units (1..256; 0 = the default 2)
 *   RT_OPT_BVH_SHAPE        the fast kernel's BVH4 over each BVH's leaf nodes, read at upload:
 *                           0 = interior levels rebuilt by the surface-area heuristic (default),
 *                           1 = the reference tree collapsed as built; the same image either way
 * Returns RT_ERR_INVALID for an unknown option or a value out of range. */
typedef enum {
    RT_OPT_TUNE = 0,
    RT_OPT_GROUP = 1,
    RT_OPT_STACK_LDS = 2,
    RT_OPT_SAMPLE_BUFFER_MB = 3,
    RT_OPT_HRPP_SLOT_BITS = 4,
    RT_OPT_LAUNCH_LOG = 5,
    RT_OPT_BVH_BUILD = 6,
    RT_OPT_GUIDE = 7,
    RT_OPT_BVH_SHAPE = 8,
    RT_OPT_COUNT = 9
} rt_option;
int rt_set_option(int option, int64_t value);
int rt_get_option(int option, int64_t* value);

/* HRPP statistics of the last RT_FLAG_HRPP render (src/hrpp.rs:91-127): for
 * predictor p (in lowering order) out[6 p + 0..5] = true-positive, false-positive
 * and no-prediction BVH calls, table entries (distinct ray hashes), predicted nodes
 * stored, insertions dropped (table or node set full). *count = predictors. */
int rt_scene_hrpp_stats(rt_scene_handle scene, uint64_t* out, uint32_t capacity, uint32_t* count);

/* Device time of the trace kernel launches issued by rt_render_launch on this
 * scene since the last reset (HIP events recorded on the launch stream around
 * each launch; waits for them). Up to 256 launches are kept between resets. */
int rt_scene_trace_time(rt_scene_handle scene, double* total_ms, uint64_t* launches, int reset);

/* Synchronous drop-in for Renderer::render minus the PPM write: renders into a
 * HOST buffer of W*H*3 floats (pixels outside the shard are left untouched). */
int rt_render(rt_scene_handle scene, const rt_camera_desc* camera,
              const rt_render_params* params, float* host_out, rt_stats* stats);

/* Camera::new (src/camera.rs:44-81) on the host: the nine fields the reference's
 * Camera stores. RT_ERR_INVALID when time0 > time1 (the reference panics in
 * Uniform::new_inclusive at the first get_ray). */
int rt_camera_new(const rt_camera_desc* args, rt_camera* out);

/* rt_render / rt_render_launch / rt_render_multi for a constructed Camera:
 * the exact arguments of Renderer::render (src/renderer.rs:42-52), which
 * borrows a built `Camera`, not its constructor arguments. The desc forms above
 * are rt_camera_new followed by these. Same results bit for bit. */
int rt_render_camera(rt_scene_handle scene, const rt_camera* camera,
                     const rt_render_params* params, float* host_out, rt_stats* stats);
int rt_render_launch_camera(rt_scene_handle scene, const rt_camera* camera,
                            const rt_render_params* params, float* d_out,
                            unsigned long long* d_segments, void* stream);
int rt_render_multi_camera(rt_scene_handle* scenes, uint32_t n, const rt_camera* camera,
                           const rt_render_params* params, float* host_out, rt_stats* stats);

/* Multi-process frame assembly (one process per GPU, no
 * collective). Rank r of n renders the 8x8 blocks b with b % n == r into a
 * full-frame device image (shard_index = r, shard_count = n);
 * rt_shard_pack copies those blocks, in block order, 64 pixel slots per block
 * (row-major in the block; slots outside the image of an edge block are left
 * unwritten), into a device buffer of rt_shard_floats(W, H, r, n) floats, which
 * the rank copies (hipMemcpyAsync) into its slot of a shared buffer at float
 * offset rt_shard_offset(W, H, r, n); rt_shard_offset(W, H, n, n) is the total.
 * rt_shard_unpack scatters all n packed shards (one device buffer, shard r at
 * its offset) back into a W*H*3 image. Both are asynchronous on `stream`.
 * Packing then unpacking every rank's shard reproduces the one-device image bit
 * for bit (pure copies). Returns 0 from the two size functions for n == 0. */
uint64_t rt_shard_floats(uint32_t width, uint32_t height, uint32_t rank, uint32_t n);
uint64_t rt_shard_offset(uint32_t width, uint32_t height, uint32_t rank, uint32_t n);
int rt_shard_pack(const float* d_image, uint32_t width, uint32_t height, uint32_t rank,
                  uint32_t n, float* d_packed, void* stream);
int rt_shard_unpack(const float* d_packed_all, uint32_t width, uint32_t height,
                    uint32_t n, float* d_image, void* stream);

/* Peer transport for that gather (device to device over xGMI, one hop), in pull form:
 * every rank r > 0 exports its packed-shard buffer once (rt_ipc_export: the
 * hipIpcMemHandle_t of the allocation holding d_ptr plus d_ptr's offset in it, in
 * RT_IPC_HANDLE_BYTES bytes the caller sends to rank 0) and rank 0 maps each of them
 * (rt_ipc_open, on its own device; unmap with rt_ipc_close). Per frame each rank r > 0
 * packs its blocks (rt_shard_pack, whose threads end with a system-scope release) and
 * synchronises its stream; after a host barrier rank 0 calls rt_shard_pull_unpack with the
 * n mapped pointers (entry 0 unused): one kernel, opening with a system-scope acquire
 * fence, reads every peer word with a system-scope load and writes ranks 1..n-1's blocks
 * into d_image, which already holds rank 0's own blocks. The visibility argument is the
 * LLVM AMDGPU memory model's, not a dispatch default. Replaces
 * renderer.rs:86-95's host-side composite of the tiles; a /dev/shm bounce stays the
 * caller's fallback where IPC is refused. rt_copy_async is a device-to-device
 * hipMemcpyAsync on `stream` (the transport's setup probe). At most 64 ranks. */
#define RT_IPC_HANDLE_BYTES 72
int rt_ipc_export(const void* d_ptr, int device, uint8_t handle[RT_IPC_HANDLE_BYTES]);
int rt_ipc_open(const uint8_t handle[RT_IPC_HANDLE_BYTES], int device, void** d_ptr);
int rt_ipc_close(void* d_ptr, int device);
int rt_copy_async(void* d_dst, const void* d_src, uint64_t bytes, void* stream);
int rt_shard_pull_unpack(const float* const* d_peer_packed, uint32_t width, uint32_t height,
                         uint32_t n, float* d_image, void* stream);

/* Scene builders restated from src/main.rs:185-829 ("random-spheres",
 * "random-moving-spheres", "two-spheres", "marble", "earth", "simple-lights",
 * "cornell", "cornell-smoke", "showcase", "bunny", "gargoyle", "igea-hrpp").
 * asset_dir holds earthmap_1024x512.rgb8 and optional OBJ meshes.
 * The returned descriptor owns its arrays; free with rt_scene_desc_free. */
int rt_scene_generate(const char* name, uint64_t seed, const char* asset_dir,
                      rt_scene_desc** out);
void rt_scene_desc_free(rt_scene_desc* desc);
/* Background of the CLI for `name` (src/main.rs:155-164). */
int rt_scene_background(const char* name, float rgb[3]);

/* Device numeric self-check (diagnostic): evaluates op on `n` inputs on the GPU.
 * op: 0 sqrt f64, 1 sqrt f32, 2 div f32, 3 rt_sinf, 4 rt_acosf, 5 rt_atan2f,
 *     6 rt_logf, 7 div f64, 8 HRPP map_float_to_hash (hrpp.rs:136-170, six bits).
 * Results are returned as doubles. */
int rt_device_numeric_eval(int op, const double* a, const double* b, double* out,
                           uint32_t n);

/* Device known answers (diagnostic): the kernel's own primitives evaluated on the GPU
 * for n cases, two floats out per case. op 0: Aabb::hit (aabb.rs:28-41) as the
 * reference-exact slab test, op 1: the same box through the fast kernel's packed
 * four-child test — in: 14 floats per case (min[3], max[3], origin[3], direction[3],
 * t_min, t_max), out: (hit 1/0, entry t); op 2: Sphere::get_uv (sphere.rs:41-46) —
 * in: p[3], out: (u, v); op 3: Sphere::hit's root (sphere.rs:49-103) — in: center[3],
 * radius, origin[3], direction[3], t_min, t_max, out: (hit 1/0, t); op 4: a cube side's
 * quotient (k - o) / d as a BVH cube leaf forms it from the ray's reciprocal (in range: RN(1/d) and
 * Markstein's correction; otherwise the division) — in: k, o, d, out: (that quotient, (k - o) / d). */
int rt_device_kat(int op, const float* in, float* out, uint32_t n);

#ifdef __cplusplus
}
#endif

#endif /* RT_H */
