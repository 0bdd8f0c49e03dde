// device_scene.hpp — layout of a lowered scene in HBM (host lowering <-> kernel).
//
// The reference walks an `Arc<dyn Hittable>` graph (src/hittable.rs:64-140).
// Here the graph is flattened once on the host (lower.cpp) into:
//   entries[]  the top-level HittableList in order (nested lists flattened,
//              Translate/RotateY chains folded into each entry), followed by
//              the boundaries of ConstantMedium entries;
//   prims      SoA float4 records for spheres / moving spheres / rects / tris;
//   nodes[]    every BVH (src/bvh.rs) as 64-byte BVH2 nodes in DFS preorder;
//   materials / textures / Perlin permutation tables / RGB8 texels.
// Everything is read-only during a render and a few MB at most, so it stays
// resident in each XCD's L2 after the first touch.
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#define RTDEV_HD __host__ __device__ inline
#else
#define RTDEV_HD inline
#endif

namespace rtdev {

struct alignas(16) f4 {
    float x, y, z, w;
};

// Child / leaf codes (BVH children, GEOM entry payloads, hit identifiers).
// bit 31 set = leaf; bits 28..30 = leaf type; bits 0..27 = index.
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kLeafSphere = 0u;   // index into sph
constexpr uint32_t kLeafMSphere = 1u;  // index into msph (3 f4 each)
constexpr uint32_t kLeafRect = 2u;     // index into rect (2 f4 each)
constexpr uint32_t kLeafCube = 3u;     // index of the first of 6 rects (cube.rs:25-74 order)
constexpr uint32_t kLeafTri = 4u;      // index into tri (3 f4 each)
constexpr uint32_t kLeafMedium = 6u;   // hit identifier of a ConstantMedium scatter point
constexpr uint32_t kChildEmpty = 0xffffffffu;  // second child of a 1-object node (bvh.rs:261-264)
constexpr uint32_t kMaxIndex = 0x0fffffffu;
constexpr uint32_t kBvhPrunable = 1u;  // wrapper-node flag: closest-hit box pruning is exact for this BVH
// BVH4 wrapper flag (rank[3], with kBvhPrunable): every leaf is a Tri (the BVH2 wrapper's
// kBvh2TriOnly below, for the fast traversal). Such a BVH is never prunable, so its slab tests
// use no delta-inflation, and the fast kernel traverses it also with a zero direction component
// (kernel.hip ray_route).
constexpr uint32_t kBvhTriOnly = 2u;
// Such a BVH also carries its leaf codes in DFS order behind its nodes (lower.cpp bvh_emit; first
// node index in the wrapper's rank[1]); kDfsPairLeft marks the left object of a two-object leaf node.
constexpr uint32_t kDfsPairLeft = 0x80000000u;
// BVH2 wrapper flag (nodes2 wrapper row 3 .w): every leaf is a Tri. Möller-Trumbore
// (triangle.rs:32-92) rejects any ray with a NaN origin or direction component (a NaN
// reaches t, and !(t > EPSILON) rejects it), so such a BVH returns no hit for that ray
// whatever its boxes do; bvh_hit_reference answers at once instead of visiting every node.
constexpr uint32_t kBvh2TriOnly = 1u;
constexpr uint32_t kBvhWidth = 4u;     // children per BVH node (collapsed from the reference BVH2)
constexpr uint32_t kBvhNodeF4 = 8u;    // f4 records per BVH node
// A BVH4 node holds either only leaves (the 1-2 leaf children of one reference
// BVH2 node, in slots 0-1) or only interior children (bvh.rs never mixes them);
// child pointers to a leaf node carry this bit so the traversal knows which rows
// to load before loading anything.
constexpr uint32_t kLeafNodeFlag = 0x40000000u;

RTDEV_HD uint32_t leaf_code(uint32_t type, uint32_t index) {
    return kLeafBit | (type << 28) | index;
}
RTDEV_HD uint32_t leaf_type(uint32_t code) { return (code >> 28) & 7u; }
RTDEV_HD uint32_t leaf_index(uint32_t code) { return code & kMaxIndex; }

enum EntryKind : uint32_t {
    kEntGeom = 0,    // payload = leaf code of one primitive / cube
    kEntBvh = 1,     // payload = root node index
    kEntMedium = 2,  // payload = boundary entry index; phase_mat, neg_inv_density
    kEntSphereRun = 3,  // payload = first sphere, pad[0] = count: consecutive top-level spheres
                        // (no transforms, consecutive sphere records), tested in list order
    kEntRectRun = 4,    // payload = first rect, pad[0] = count: the same for rectangles (walls, lights)
};

constexpr int kMaxTransforms = 3;

// One top-level object (80 bytes). Transform ops are listed outer -> inner:
//   w == 0: Translate by (x, y, z)   (instance.rs:32-43)
//   w == 1: RotateY, x = sin, y = cos (instance.rs:114-143)
struct alignas(16) DevEntry {
    uint32_t kind;
    uint32_t payload;
    uint32_t ntf;
    uint32_t phase_mat;
    float neg_inv_density;
    uint32_t pad[3];
    f4 tf[kMaxTransforms];
};
static_assert(sizeof(DevEntry) == 80, "DevEntry layout");

enum MatKind : uint32_t { kMatLambertian = 0, kMatMetal = 1, kMatDielectric = 2, kMatLight = 3, kMatIsotropic = 4 };
constexpr uint32_t kMatNeedsUV = 1u;  // some texture of the material reads (u, v): an ImageTexture
struct alignas(16) DevMaterial {
    uint32_t kind;
    uint32_t tex;
    float fuzz;
    float ior;
    float albedo[3];
    uint32_t flags;
};
static_assert(sizeof(DevMaterial) == 32, "DevMaterial layout");

enum TexKind : uint32_t { kTexSolid = 0, kTexChecker = 1, kTexMarble = 2, kTexImage = 3 };
// checker: a = even, b = odd; marble: a = first of 9 permutation tables
// (source, then distortion seeds 0..7); image: a = texel byte offset, b = w, c = h.
struct alignas(16) DevTexture {
    uint32_t kind;
    uint32_t a, b, c;
    float color[3];
    float scale;
};
static_assert(sizeof(DevTexture) == 32, "DevTexture layout");

// Record layouts (f4 units):
//   sph  : (cx, cy, cz, r)                       + sph_mat[] (u32)
//   msph : (c0, r) (c1 - c0, t0) (t1 - t0, mat, 0, 0)     moving_sphere.rs:47-51
//   rect : (k, a0, a1, b0) (b1, axis, mat, 0)  axis 0 = XY, 1 = XZ, 2 = YZ
//   tri  : (v0, mat) (v1 - v0, 0) (v2 - v0, 0)           triangle.rs:44-45
//   node : 128 B BVH4 node (kBvhNodeF4 f4): (min.x[4]) (min.y[4]) (min.z[4])
//          (max.x[4]) (max.y[4]) (max.z[4]) (child[4]) (rank[4]); child = node
//          index (| kLeafNodeFlag for a leaf node), leaf code or kChildEmpty; a leaf slot's box is the leaf's own
//          bounding box (used only by the conservative leaf reject), its rank the
//          leaf's DFS ordinal in the reference BVH2. A leaf node's spheres are repeated
//          in the free lanes 2 / 3 of rows 0, 1, 2, 6 (lower.cpp bvh_emit put).
//          Each BVH starts with a wrapper
//          node whose slot 0 is the root; the wrapper's rank[3] holds kBvhPrunable
//          when every leaf is a Sphere/Rect/Cube, its rank[2] the BVH2 wrapper.
//   node2: 64 B reference BVH2 node: (Lmin, Lmax.x) (Lmax.yz, Rmin.xy) (Rmin.z,
//          Rmax) (left, right, 0, 0), DFS preorder behind a wrapper (child 0 = root;
//          row 3 .z = HRPP predictor id, .w = kBvh2TriOnly).
// One HRPP table slot (32 B): a 48-bit ray hash (hrpp.rs:172-193; ~0 = empty) and
// up to kHrppIds predicted leaf nodes (the reference keeps an unbounded set; the
// paper's implementation, which hrpp.rs:62 cites, keeps 5).
constexpr uint32_t kHrppIds = 6;
constexpr uint32_t kHrppMaxPredictors = 8;
struct HrppSlot {
    unsigned long long key;
    uint32_t ids[kHrppIds];
};

struct DevScene {
    const DevEntry* entries;
    const f4* sph;
    const uint32_t* sph_mat;
    const f4* msph;
    const f4* rect;
    const f4* tri;
    const f4* nodes;
    const f4* nodes2;  // the reference BVH2 trees (bvh_hit_reference)
    const DevMaterial* mats;
    const DevTexture* texs;
    const uint8_t* perm;
    const uint8_t* texels;
    uint32_t num_top;
    uint32_t num_entries;
    uint32_t stack_depth;  // LDS traversal stack entries per lane
    uint32_t perm_bytes;   // size of perm[] (staged in LDS when it fits)
    // HRPP experiment (RT_FLAG_HRPP; null otherwise). Predictor p (1-based, in the
    // BVH2 wrapper's row 3 .z) owns table slots [(p - 1) << hrpp_bits, p << hrpp_bits).
    HrppSlot* hrpp_tab;
    const unsigned long long* hrpp_keys;  // sorted (wrapper2 << 32 | leaf code)
    const uint32_t* hrpp_vals;            // -> wrapper-format record of the leaf node
    unsigned long long* hrpp_stats;       // per predictor: tp, fp, np, dropped
    uint32_t* hrpp_cnt;                   // per-wave LDS counters (set in the kernel)
    uint32_t hrpp_bits, hrpp_nkeys, hrpp_npred;
    uint32_t num_nodes2;  // BVH2 records (the audit build bounds-checks every visited index)
    // Deep BVHs (instances with kFDeep): stack entries past stack_depth live in HBM,
    // stack_spill[((wave * spill_depth + entry - stack_depth) * 64 + lane) * 2 + {node, t}]
    uint32_t* stack_spill;
    uint32_t spill_depth;
    uint32_t num_nodes;   // BVH4 nodes (the audit build bounds-checks every visited index)
    // Every rect / cube-side coordinate is +0 or of magnitude in [2^-20, 2^20] (set at upload): a
    // cube leaf's side quotients may then come from the ray's reciprocals (kernel.hip div_rn_safe).
    uint32_t rect_rcp_ok;
    // The first top-level ConstantMedium when its boundary is one sphere and every entry before it
    // is a sphere / moving sphere / rect / cube / sphere run or a prunable, translated-only BVH
    // (kernel.hip medium_first_estimate); ~0 otherwise.
    uint32_t mb_entry;
    // Material and texture records (32 B each) of a small scene, in that order; the flat-list
    // preset's fast kernel stages them in LDS when the launch sets mt_lds (their byte size).
    uint32_t num_mats, num_texs, mt_lds;
};

// Camera::new (camera.rs:44-81) evaluated on the host.
struct DevCamera {
    float origin[3], horizontal[3], vertical[3], llc[3], u[3], v[3];
    float lens_radius, time_low, time_scale;
};

struct DevParams {
    uint32_t width, height, spp, max_depth;
    uint32_t seed_lo, seed_hi, sample_base;
    uint32_t shard_index, shard_count, blocks_x, num_blocks;
    uint32_t flags;
    float bg[3];
    float prune_delta;  // box inflation for closest-hit pruning ("exact pruning")
    uint32_t tune;      // kMode* traversal switches from RT_TUNE (diagnostics)
    uint32_t spp_div;   // divisor of the final average (rt_render_params.spp_total or spp)
};

}  // namespace rtdev
