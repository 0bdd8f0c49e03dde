// lower.hpp — host-side lowering of the scene IR (include/rt.h) to the device
// layout (device_scene.hpp), plus the host halves of Camera::new and the
// split-axis / Perlin random streams that must match the oracle bit for bit.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rt.h"
#include "device_scene.hpp"

namespace rthost {

struct HostScene {
    std::vector<rtdev::DevEntry> entries;
    uint32_t num_top = 0;
    std::vector<rtdev::f4> sph;
    std::vector<uint32_t> sph_mat;
    std::vector<rtdev::f4> msph, rect, tri, nodes, nodes2;
    std::vector<rtdev::DevMaterial> mats;
    std::vector<rtdev::DevTexture> texs;
    std::vector<uint8_t> perm, texels;
    uint32_t max_bvh_depth = 0;  // internal levels of the deepest BVH (reference BVH2)
    bool bvh_rect_msph = false;  // some BVH has rect or moving-sphere leaves (the fast kernel's kFLeafRM)
    uint32_t max_stack = 1;      // BVH4 traversal stack entries (2 words) per lane
    uint32_t max_stack_ref = 1;  // the same for the BVH2 replay (reference kernel)
    // Upper bound on |coordinate| of any primitive in any instance frame plus the
    // translations applied to reach it (bounds ray lengths for the pruning margin).
    float coord_bound = 0.0f;
    // HRPP (Bvh::with_predictor BVHs): count, and the sorted map
    // (BVH2 wrapper << 32 | leaf code) -> wrapper-format record of its leaf node.
    uint32_t num_predictors = 0;
    std::vector<uint64_t> hrpp_keys;
    std::vector<uint32_t> hrpp_vals;
    uint64_t bytes() const;
};

// Bvh::new's leaf order computed outside the host recursion (the device builder,
// bvh_build.hip): fills order[n] with the item indices in the order the reference
// recursion leaves them (bvh.rs:249-333), from keys[3 * i + axis] =
// bounding_box(0, 0).min of item i and the BVH's split-axis seed.
struct BvhOrderer {
    uint32_t min_items;  // BVHs with fewer items are ordered by the host recursion
    int (*fn)(void* ctx, const float* keys, uint32_t n, uint64_t seed, uint32_t* order, std::string* err);
    void* ctx;
};

// The tree shape of the fast kernel's BVH4 (rt.h RT_OPT_BVH_SHAPE): rebuilt by SAH over the reference
// tree's leaf nodes (0, the default), or the reference tree collapsed as built (1).
constexpr int kBvhShapeSah = 0, kBvhShapeReference = 1;
// Returns RT_OK or a negative rt_status with a message in *err.
int lower_scene(const rt_scene_desc* desc, HostScene* out, std::string* err, const BvhOrderer* orderer = nullptr,
                int bvh_shape = kBvhShapeSah);

// BvhOrderer::fn backed by rt_bvh_build_order on device *(int*)ctx (bvh_build.hip).
int device_bvh_order(void* ctx, const float* keys, uint32_t n, uint64_t seed, uint32_t* order, std::string* err);

// Camera::new (src/camera.rs:44-81); returns RT_ERR_INVALID when time0 > time1
// (the reference panics in UniformFloat::new_inclusive).
int camera_new(const rt_camera_desc* args, rt_camera* out, std::string* err);
// The kernel's copy of a constructed Camera (src/camera.rs:6-27) plus the
// UniformFloat::new_inclusive scale of gen_range(time_start..=time_end) (camera.rs:104).
int camera_device(const rt_camera* cam, rtdev::DevCamera* out, std::string* err);
// camera_new followed by camera_device.
int camera_basis(const rt_camera_desc* cam, rtdev::DevCamera* out, std::string* err);

// Philox4x32-10 (Random123), host copy used by the split-axis stream.
void philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

// noise 0.8.2 PermutationTable::new(seed) restatement (XorShift128 + rand 0.7 shuffle).
void perlin_permutation(uint32_t seed, uint8_t out[256]);

}  // namespace rthost
