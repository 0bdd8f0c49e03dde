// scene_builder.hpp — host-side mirror of the reference's constructor surface
// (Sphere::new, Lambertian::from_color, Bvh::new, RotateY::new, ...), emitting
// the scene IR of include/rt.h. Each method is one reference constructor.
#pragma once
#include <stdint.h>

#include <initializer_list>
#include <string>
#include <vector>

#include "../../include/rt.h"

namespace rthost {

struct Vec3 {
    float x, y, z;
};

// hittable.rs:84-98 — a HittableList under construction (node indices).
struct HittableList {
    std::vector<int32_t> objects;
    void add(int obj) { objects.push_back(obj); }
};

// Scene-generation stream (replaces the thread_rng draws of src/main.rs).
class SceneRng {
   public:
    explicit SceneRng(uint64_t seed);
    uint32_t next_u32();
    uint64_t next_u64();
    float std01();                      // rand::random::<f32>()
    float range(float low, float high); // rng.gen_range(low..high)

   private:
    uint32_t key_[2];
    uint32_t block_ = 0, buf_[4] = {0, 0, 0, 0};
    int idx_ = 4;
};

class SceneBuilder {
   public:
    // textures (src/textures)
    int solid(Vec3 c);
    int checker(float scale, int even, int odd);
    int checker_from_color(float scale, Vec3 even, Vec3 odd);
    int marble(float scale, uint32_t perlin_seed);
    int image(const uint8_t* rgb, uint32_t w, uint32_t h);
    // materials (src/materials)
    int lambertian(int tex);
    int lambertian_from_color(Vec3 c);
    int metal(Vec3 albedo, float fuzz);
    int dielectric(float ior);
    int diffuse_light(int tex);
    int diffuse_light_from_color(Vec3 c);
    int isotropic(int tex);
    // hittables (src/geometry, src/hittable.rs, src/bvh.rs)
    int sphere(Vec3 c, float r, int mat);
    int moving_sphere(Vec3 c0, Vec3 c1, float t0, float t1, float r, int mat);
    int xy_rect(float x0, float x1, float y0, float y1, float k, int mat);
    int xz_rect(float x0, float x1, float z0, float z1, float k, int mat);
    int yz_rect(float y0, float y1, float z0, float z1, float k, int mat);
    int cube(Vec3 mn, Vec3 mx, int mat);
    int tri(Vec3 p0, Vec3 p1, Vec3 p2, int mat);
    int list(const HittableList& l);
    // predictor: Bvh::with_predictor (bvh.rs:69-80) rather than Bvh::new
    int bvh(const HittableList& l, float t0, float t1, uint64_t axis_seed, bool predictor = false);
    int translate(int child, Vec3 d);
    int rotate_y(int child, float degrees);
    int constant_medium(int boundary, float density, int tex);
    int constant_medium_from_color(int boundary, float density, Vec3 c);

    // Moves the arrays into a heap descriptor freed by free_desc / rt_scene_desc_free.
    rt_scene_desc* finish(int world_list);
    static void free_desc(rt_scene_desc* d);

    std::vector<rt_node> nodes;
    std::vector<int32_t> items;
    std::vector<uint8_t> images;

   private:
    int add(uint32_t kind, std::initializer_list<float> f, int r0 = -1, int r1 = -1, int r2 = -1, uint64_t seed = 0);
};

int generate_scene(const std::string& name, uint64_t seed, const std::string& asset_dir, rt_scene_desc** out);
int scene_background(const std::string& name, float rgb[3]);

}  // namespace rthost
