// scenes.cpp — the reference's sample scenes (src/main.rs:185-829) restated as
// deterministic generators that emit the scene IR of include/rt.h.
//
// The reference draws scene randomness from OS-seeded thread_rng; here one
// Philox4x32-10 stream keyed by the caller's seed feeds the same draws in the
// same order, through the same rand 0.8.5 f32 constructions (Standard,
// gen_range). Each BVH gets its split-axis stream seed from this stream at the
// point where the reference calls Bvh::new / Bvh::with_predictor.
//
// HRPP predictors (Bvh::with_predictor, src/main.rs:586, 679, 824) are marked
// on their BVH nodes (ref[1] = 1); renders use the exact traversal (bvh.rs:212-217)
// unless RT_FLAG_HRPP asks for the prediction experiment.
#include <math.h>
#include <stddef.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "../../include/rt_numeric_spec.h"
#include "common.hpp"
#include "lower.hpp"
#include "scene_builder.hpp"

namespace rthost {

// ---------------------------------------------------------------------------
// SceneRng
// ---------------------------------------------------------------------------
SceneRng::SceneRng(uint64_t seed) {
    key_[0] = (uint32_t)seed;
    key_[1] = (uint32_t)(seed >> 32);
}
uint32_t SceneRng::next_u32() {
    if (idx_ == 4) {
        // counter (block, 0xffffffff, 0xffffffff, 1): disjoint from every pixel stream
        uint32_t ctr[4] = {block_++, 0xffffffffu, 0xffffffffu, 1u};
        philox4x32_10(ctr, key_, buf_);
        idx_ = 0;
    }
    return buf_[idx_++];
}
uint64_t SceneRng::next_u64() {
    uint64_t lo = next_u32();
    uint64_t hi = next_u32();
    return lo | (hi << 32);
}
float SceneRng::std01() { return (1.0f / 16777216.0f) * (float)(next_u32() >> 8); }
float SceneRng::range(float low, float high) {  // UniformFloat::sample_single
    float scale = high - low;
    for (;;) {
        float v01 = rt_spec_bits_f32((next_u32() >> 9) | 0x3f800000u) - 1.0f;
        float res = v01 * scale + low;
        if (res < high) return res;
        scale = rt_spec_bits_f32(rt_spec_f32_bits(scale) - 1u);
    }
}

// ---------------------------------------------------------------------------
// SceneBuilder
// ---------------------------------------------------------------------------
int SceneBuilder::add(uint32_t kind, std::initializer_list<float> f, int r0, int r1, int r2, uint64_t seed) {
    rt_node n;
    memset(&n, 0, sizeof n);
    n.kind = kind;
    n.ref[0] = r0;
    n.ref[1] = r1;
    n.ref[2] = r2;
    int i = 0;
    for (float v : f) {
        if (i < 12) n.f[i++] = v;
    }
    n.seed = seed;
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}
int SceneBuilder::solid(Vec3 c) { return add(RT_TEX_SOLID, {c.x, c.y, c.z}); }
int SceneBuilder::checker(float scale, int even, int odd) { return add(RT_TEX_CHECKER, {scale}, even, odd); }
int SceneBuilder::checker_from_color(float scale, Vec3 even, Vec3 odd) {
    int e = solid(even);
    int o = solid(odd);
    return checker(scale, e, o);
}
int SceneBuilder::marble(float scale, uint32_t seed) { return add(RT_TEX_MARBLE, {scale}, -1, -1, -1, seed); }
int SceneBuilder::image(const uint8_t* rgb, uint32_t w, uint32_t h) {
    uint64_t off = images.size();
    images.insert(images.end(), rgb, rgb + (size_t)w * h * 3u);
    return add(RT_TEX_IMAGE, {}, (int)w, (int)h, -1, off);
}
int SceneBuilder::lambertian(int tex) { return add(RT_MAT_LAMBERTIAN, {}, tex); }
int SceneBuilder::lambertian_from_color(Vec3 c) { return lambertian(solid(c)); }
int SceneBuilder::metal(Vec3 albedo, float fuzz) { return add(RT_MAT_METAL, {albedo.x, albedo.y, albedo.z, fuzz}); }
int SceneBuilder::dielectric(float ior) { return add(RT_MAT_DIELECTRIC, {ior}); }
int SceneBuilder::diffuse_light(int tex) { return add(RT_MAT_DIFFUSE_LIGHT, {}, tex); }
int SceneBuilder::diffuse_light_from_color(Vec3 c) { return diffuse_light(solid(c)); }
int SceneBuilder::isotropic(int tex) { return add(RT_MAT_ISOTROPIC, {}, tex); }
int SceneBuilder::sphere(Vec3 c, float r, int mat) { return add(RT_OBJ_SPHERE, {c.x, c.y, c.z, r}, mat); }
int SceneBuilder::moving_sphere(Vec3 c0, Vec3 c1, float t0, float t1, float r, int mat) {
    return add(RT_OBJ_MOVING_SPHERE, {c0.x, c0.y, c0.z, c1.x, c1.y, c1.z, t0, t1, r}, mat);
}
int SceneBuilder::xy_rect(float x0, float x1, float y0, float y1, float k, int mat) {
    return add(RT_OBJ_XY_RECT, {x0, x1, y0, y1, k}, mat);
}
int SceneBuilder::xz_rect(float x0, float x1, float z0, float z1, float k, int mat) {
    return add(RT_OBJ_XZ_RECT, {x0, x1, z0, z1, k}, mat);
}
int SceneBuilder::yz_rect(float y0, float y1, float z0, float z1, float k, int mat) {
    return add(RT_OBJ_YZ_RECT, {y0, y1, z0, z1, k}, mat);
}
int SceneBuilder::cube(Vec3 mn, Vec3 mx, int mat) { return add(RT_OBJ_CUBE, {mn.x, mn.y, mn.z, mx.x, mx.y, mx.z}, mat); }
int SceneBuilder::tri(Vec3 p0, Vec3 p1, Vec3 p2, int mat) {
    return add(RT_OBJ_TRI, {p0.x, p0.y, p0.z, p1.x, p1.y, p1.z, p2.x, p2.y, p2.z}, mat);
}
int SceneBuilder::list(const HittableList& l) {
    int first = (int)items.size();
    items.insert(items.end(), l.objects.begin(), l.objects.end());
    return add(RT_OBJ_LIST, {}, first, (int)l.objects.size());
}
int SceneBuilder::bvh(const HittableList& l, float t0, float t1, uint64_t axis_seed, bool predictor) {
    int li = list(l);
    return add(RT_OBJ_BVH, {t0, t1}, li, predictor ? 1 : -1, -1, axis_seed);
}
int SceneBuilder::translate(int child, Vec3 d) { return add(RT_OBJ_TRANSLATE, {d.x, d.y, d.z}, child); }
int SceneBuilder::rotate_y(int child, float degrees) { return add(RT_OBJ_ROTATE_Y, {degrees}, child); }
int SceneBuilder::constant_medium(int boundary, float density, int tex) {
    return add(RT_OBJ_CONSTANT_MEDIUM, {density}, boundary, tex);
}
int SceneBuilder::constant_medium_from_color(int boundary, float density, Vec3 c) {
    return constant_medium(boundary, density, solid(c));
}

namespace {
struct OwnedDesc {  // rt_scene_desc first, so the descriptor pointer frees the owner
    rt_scene_desc desc;
    std::vector<rt_node> nodes;
    std::vector<int32_t> items;
    std::vector<uint8_t> images;
};
}  // namespace

rt_scene_desc* SceneBuilder::finish(int world_list) {
    OwnedDesc* o = new OwnedDesc();
    o->nodes = std::move(nodes);
    o->items = std::move(items);
    o->images = std::move(images);
    memset(&o->desc, 0, sizeof o->desc);
    o->desc.nodes = o->nodes.data();
    o->desc.num_nodes = (uint32_t)o->nodes.size();
    o->desc.world = world_list;
    o->desc.list_items = o->items.data();
    o->desc.num_list_items = (uint32_t)o->items.size();
    o->desc.image_data = o->images.empty() ? nullptr : o->images.data();
    o->desc.image_bytes = o->images.size();
    return &o->desc;
}
void SceneBuilder::free_desc(rt_scene_desc* d) { delete reinterpret_cast<OwnedDesc*>(d); }

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
namespace {

Vec3 vec3(float x, float y, float z) { return Vec3{x, y, z}; }
Vec3 operator+(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
Vec3 operator-(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
Vec3 operator*(Vec3 a, Vec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
float length(Vec3 a) { return __builtin_sqrtf((a.x * a.x + a.y * a.y) + a.z * a.z); }

// materials/utils.rs:48-63
Vec3 random_color(SceneRng& r) {
    float x = r.std01();
    float y = r.std01();
    float z = r.std01();
    return vec3(x, y, z);
}
Vec3 random_color_range(SceneRng& r, float mn, float mx) {
    float lo = mn > 0.0f ? mn : 0.0f;  // f32::max(min, 0.0)
    float hi = 1.0f < mx ? 1.0f : mx;  // f32::min(1.0, max)
    float x = r.range(lo, hi);
    float y = r.range(lo, hi);
    float z = r.range(lo, hi);
    return vec3(x, y, z);
}

bool read_file(const std::string& path, std::vector<uint8_t>* out) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (n < 0) {
        fclose(f);
        return false;
    }
    out->resize((size_t)n);
    size_t got = n ? fread(out->data(), 1, (size_t)n, f) : 0;
    fclose(f);
    return got == (size_t)n;
}

int load_earth(SceneBuilder& b, const std::string& dir, int* tex) {
    std::vector<uint8_t> rgb;
    std::string p = dir + "/earthmap_1024x512.rgb8";
    if (!read_file(p, &rgb) || rgb.size() != 1024u * 512u * 3u)
        return set_error(RT_ERR_IO, "missing or short " + p + " (decoded images/earthmap.jpg)");
    *tex = b.image(rgb.data(), 1024, 512);
    return RT_OK;
}

// src/main.rs:185-251 (random_spheres) / 253-321 (random_moving_spheres)
int random_spheres(SceneBuilder& b, SceneRng& rng, bool moving, bool use_bvh, int* world) {
    HittableList w;
    int ground = b.lambertian(b.checker_from_color(10.0f, vec3(0.2f, 0.3f, 0.1f), vec3(0.9f, 0.9f, 0.9f)));
    w.add(b.sphere(vec3(0.0f, -1000.0f, 0.0f), 1000.0f, ground));
    for (int a = -11; a < 11; ++a) {
        for (int bb = -11; bb < 11; ++bb) {
            float choose_mat = rng.std01();
            float cx = (float)a + 0.9f * rng.std01();
            float cz = (float)bb + 0.9f * rng.std01();
            Vec3 center = vec3(cx, 0.2f, cz);
            if (length(center - vec3(4.0f, 0.2f, 0.0f)) > 0.9f) {
                int mat;
                if (choose_mat < 0.8f) {
                    Vec3 c1 = random_color(rng);
                    Vec3 c2 = random_color(rng);
                    mat = b.lambertian_from_color(c1 * c2);
                } else if (choose_mat < 0.95f) {
                    Vec3 albedo = random_color_range(rng, 0.5f, 1.0f);
                    float fuzz = rng.std01() * 0.5f;
                    mat = b.metal(albedo, fuzz);
                } else {
                    mat = b.dielectric(1.5f);
                }
                if (moving) {
                    Vec3 center_end = center + vec3(0.0f, rng.std01() * 0.5f, 0.0f);
                    w.add(b.moving_sphere(center, center_end, 0.0f, 1.0f, 0.2f, mat));
                } else {
                    w.add(b.sphere(center, 0.2f, mat));
                }
            }
        }
    }
    w.add(b.sphere(vec3(0.0f, 1.0f, 0.0f), 1.0f, b.dielectric(1.5f)));
    w.add(b.sphere(vec3(-4.0f, 1.0f, 0.0f), 1.0f, b.lambertian_from_color(vec3(0.4f, 0.2f, 0.1f))));
    w.add(b.sphere(vec3(4.0f, 1.0f, 0.0f), 1.0f, b.metal(vec3(0.7f, 0.6f, 0.5f), 0.0f)));
    uint64_t axis_seed = rng.next_u64();
    if (!use_bvh) {  // BASELINE C2: the same spheres as a plain ordered list (no Bvh::new)
        *world = b.list(w);
        return RT_OK;
    }
    int bvh = b.bvh(w, 0.0f, 1.0f, axis_seed);
    HittableList world_list;
    world_list.add(bvh);
    *world = b.list(world_list);
    return RT_OK;
}

// src/main.rs:323-343
int two_spheres(SceneBuilder& b, int* world) {
    HittableList w;
    int checker = b.lambertian(b.checker_from_color(10.0f, vec3(0.2f, 0.3f, 0.1f), vec3(0.9f, 0.9f, 0.9f)));
    w.add(b.sphere(vec3(0.0f, -10.0f, 0.0f), 10.0f, checker));
    w.add(b.sphere(vec3(0.0f, 10.0f, 0.0f), 10.0f, checker));
    *world = b.list(w);
    return RT_OK;
}

// src/main.rs:345-360
int two_marble_spheres(SceneBuilder& b, SceneRng& rng, int* world) {
    HittableList w;
    int marble = b.marble(4.0f, rng.next_u32());
    w.add(b.sphere(vec3(0.0f, -1000.0f, 0.0f), 1000.0f, b.lambertian(marble)));
    w.add(b.sphere(vec3(0.0f, 2.0f, 0.0f), 2.0f, b.lambertian(marble)));
    *world = b.list(w);
    return RT_OK;
}

// src/main.rs:368-375
int earth(SceneBuilder& b, const std::string& dir, int* world) {
    int tex;
    int rc = load_earth(b, dir, &tex);
    if (rc) return rc;
    HittableList w;
    w.add(b.sphere(vec3(0.0f, 0.0f, 0.0f), 2.0f, b.lambertian(tex)));
    *world = b.list(w);
    return RT_OK;
}

// src/main.rs:377-401
int simple_lights(SceneBuilder& b, SceneRng& rng, int* world) {
    HittableList w;
    int marble = b.marble(4.0f, rng.next_u32());
    w.add(b.sphere(vec3(0.0f, -1000.0f, 0.0f), 1000.0f, b.lambertian(marble)));
    w.add(b.sphere(vec3(0.0f, 2.0f, 0.0f), 2.0f, b.lambertian(marble)));
    int light = b.diffuse_light_from_color(vec3(4.0f, 4.0f, 4.0f));
    w.add(b.xy_rect(3.0f, 5.0f, 1.0f, 3.0f, -2.0f, light));
    w.add(b.sphere(vec3(0.0f, 7.0f, 0.0f), 2.0f, light));
    *world = b.list(w);
    return RT_OK;
}

// src/main.rs:403-475 (cornell_box) and 477-557 (cornell_smoke)
int cornell(SceneBuilder& b, bool smoke, int* world) {
    HittableList w;
    int red = b.lambertian_from_color(vec3(0.65f, 0.05f, 0.05f));
    int white = b.lambertian_from_color(vec3(0.73f, 0.73f, 0.73f));
    int green = b.lambertian_from_color(vec3(0.12f, 0.45f, 0.15f));
    int light = b.diffuse_light_from_color(smoke ? vec3(7.0f, 7.0f, 7.0f) : vec3(15.0f, 15.0f, 15.0f));
    w.add(b.yz_rect(0.0f, 555.0f, 0.0f, 555.0f, 555.0f, green));
    w.add(b.yz_rect(0.0f, 555.0f, 0.0f, 555.0f, 0.0f, red));
    if (smoke) w.add(b.xz_rect(113.0f, 443.0f, 127.0f, 432.0f, 554.0f, light));
    else w.add(b.xz_rect(213.0f, 343.0f, 227.0f, 332.0f, 554.0f, light));
    w.add(b.xz_rect(0.0f, 555.0f, 0.0f, 555.0f, 0.0f, white));
    w.add(b.xz_rect(0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
    w.add(b.xy_rect(0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
    int box1 = b.cube(vec3(0.0f, 0.0f, 0.0f), vec3(165.0f, 330.0f, 165.0f), white);
    box1 = b.translate(b.rotate_y(box1, 15.0f), vec3(265.0f, 0.0f, 295.0f));
    int box2 = b.cube(vec3(0.0f, 0.0f, 0.0f), vec3(165.0f, 165.0f, 165.0f), white);
    box2 = b.translate(b.rotate_y(box2, -18.0f), vec3(130.0f, 0.0f, 65.0f));
    if (smoke) {
        w.add(b.constant_medium_from_color(box1, 0.01f, vec3(0.0f, 0.0f, 0.0f)));
        w.add(b.constant_medium_from_color(box2, 0.01f, vec3(1.0f, 1.0f, 1.0f)));
    } else {
        w.add(box1);
        w.add(box2);
    }
    *world = b.list(w);
    return RT_OK;
}

// src/main.rs:559-686 (both BVHs carry predictors, used only under RT_FLAG_HRPP)
int showcase(SceneBuilder& b, SceneRng& rng, const std::string& dir, int* world) {
    HittableList boxes;
    int ground = b.lambertian_from_color(vec3(0.48f, 0.83f, 0.53f));
    const int boxes_per_side = 20;
    for (int i = 0; i < boxes_per_side; ++i) {
        for (int j = 0; j < boxes_per_side; ++j) {
            float w = 100.0f;
            float x0 = -1000.0f + (float)i * w;
            float z0 = -1000.0f + (float)j * w;
            float y0 = 0.0f;
            float x1 = x0 + w;
            float y1 = rng.range(1.0f, 101.0f);
            float z1 = z0 + w;
            boxes.add(b.cube(vec3(x0, y0, z0), vec3(x1, y1, z1), ground));
        }
    }
    HittableList wl;
    wl.add(b.bvh(boxes, 0.0f, 1.0f, rng.next_u64(), true));  // Bvh::with_predictor, main.rs:586-591
    int light = b.diffuse_light_from_color(vec3(7.0f, 7.0f, 7.0f));
    wl.add(b.xz_rect(123.0f, 423.0f, 147.0f, 412.0f, 554.0f, light));
    Vec3 center1 = vec3(400.0f, 400.0f, 200.0f);
    Vec3 center2 = center1 + vec3(30.0f, 0.0f, 0.0f);
    int ms_mat = b.lambertian_from_color(vec3(0.7f, 0.3f, 0.1f));
    wl.add(b.moving_sphere(center1, center2, 0.0f, 1.0f, 50.0f, ms_mat));
    wl.add(b.sphere(vec3(260.0f, 150.0f, 45.0f), 50.0f, b.dielectric(1.5f)));
    wl.add(b.sphere(vec3(0.0f, 150.0f, 145.0f), 50.0f, b.metal(vec3(0.8f, 0.8f, 0.9f), 1.0f)));
    int boundary = b.sphere(vec3(360.0f, 150.0f, 145.0f), 70.0f, b.dielectric(1.5f));
    wl.add(boundary);
    wl.add(b.constant_medium_from_color(boundary, 0.2f, vec3(0.2f, 0.4f, 0.9f)));
    int boundary2 = b.sphere(vec3(0.0f, 0.0f, 0.0f), 5000.0f, b.dielectric(1.5f));
    wl.add(b.constant_medium_from_color(boundary2, 0.0001f, vec3(1.0f, 1.0f, 1.0f)));
    int earth_tex;
    int rc = load_earth(b, dir, &earth_tex);
    if (rc) return rc;
    wl.add(b.sphere(vec3(400.0f, 200.0f, 400.0f), 100.0f, b.lambertian(earth_tex)));
    int perlin = b.marble(0.1f, rng.next_u32());
    wl.add(b.sphere(vec3(220.0f, 280.0f, 300.0f), 80.0f, b.lambertian(perlin)));
    HittableList spheres;
    int white = b.lambertian_from_color(vec3(0.73f, 0.73f, 0.73f));
    for (int i = 0; i < 1000; ++i) {
        const float max_val = 165.0f;
        float rx = rng.range(0.0f, max_val);
        float ry = rng.range(0.0f, max_val);
        float rz = rng.range(0.0f, max_val);
        spheres.add(b.sphere(vec3(rx, ry, rz), 10.0f, white));
    }
    int sb = b.bvh(spheres, 0.0f, 1.0f, rng.next_u64(), true);  // main.rs:679
    wl.add(b.translate(b.rotate_y(sb, 15.0f), vec3(-100.0f, 270.0f, 395.0f)));
    *world = b.list(wl);
    return RT_OK;
}

// src/main.rs:688-743
HittableList cornell_boundaries(SceneBuilder& b) {
    HittableList w;
    int red = b.lambertian_from_color(vec3(0.65f, 0.05f, 0.05f));
    int white = b.lambertian_from_color(vec3(0.73f, 0.73f, 0.73f));
    int green = b.lambertian_from_color(vec3(0.12f, 0.45f, 0.15f));
    int light = b.diffuse_light_from_color(vec3(15.0f, 15.0f, 15.0f));
    w.add(b.xz_rect(200.0f, 356.0f, 200.0f, 359.0f, 554.0f, light));
    w.add(b.yz_rect(0.0f, 555.0f, 0.0f, 555.0f, 555.0f, green));
    w.add(b.yz_rect(0.0f, 555.0f, 0.0f, 555.0f, 0.0f, red));
    w.add(b.xz_rect(0.0f, 555.0f, 0.0f, 555.0f, 0.0f, white));
    w.add(b.xz_rect(0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
    w.add(b.xy_rect(0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
    return w;
}

// Stand-in for models/bunny_2000_scale.obj (a Git-LFS pointer in the reference
// checkout): icosphere subdivided 5x (20,480 triangles), radially displaced by a
// smooth deterministic field, ~90 units in radius, just above y = 0.
std::vector<float> synthetic_mesh(int level) {
    std::vector<double> v;
    auto addv = [&](double x, double y, double z) {
        double l = sqrt(x * x + y * y + z * z);
        v.push_back(x / l);
        v.push_back(y / l);
        v.push_back(z / l);
        return (int)(v.size() / 3 - 1);
    };
    const double t = (1.0 + sqrt(5.0)) / 2.0;
    addv(-1, t, 0); addv(1, t, 0); addv(-1, -t, 0); addv(1, -t, 0);
    addv(0, -1, t); addv(0, 1, t); addv(0, -1, -t); addv(0, 1, -t);
    addv(t, 0, -1); addv(t, 0, 1); addv(-t, 0, -1); addv(-t, 0, 1);
    std::vector<int> f = {0, 11, 5, 0, 5, 1, 0, 1, 7, 0, 7, 10, 0, 10, 11, 1, 5, 9, 5, 11, 4, 11, 10, 2, 10, 7, 6, 7, 1, 8,
                          3, 9, 4, 3, 4, 2, 3, 2, 6, 3, 6, 8, 3, 8, 9, 4, 9, 5, 2, 4, 11, 6, 2, 10, 8, 6, 7, 9, 8, 1};
    for (int l = 0; l < level; ++l) {
        std::map<std::pair<int, int>, int> mid;
        auto midpoint = [&](int a, int c) {
            std::pair<int, int> key = a < c ? std::make_pair(a, c) : std::make_pair(c, a);
            auto it = mid.find(key);
            if (it != mid.end()) return it->second;
            int m = addv(v[3 * a] + v[3 * c], v[3 * a + 1] + v[3 * c + 1], v[3 * a + 2] + v[3 * c + 2]);
            mid[key] = m;
            return m;
        };
        std::vector<int> nf;
        for (size_t i = 0; i < f.size(); i += 3) {
            int a = f[i], bb = f[i + 1], c = f[i + 2];
            int ab = midpoint(a, bb), bc = midpoint(bb, c), ca = midpoint(c, a);
            int tri[12] = {a, ab, ca, bb, bc, ab, c, ca, bc, ab, bc, ca};
            nf.insert(nf.end(), tri, tri + 12);
        }
        f.swap(nf);
    }
    std::vector<float> out;
    out.reserve(f.size() * 3);
    for (int idx : f) {
        double x = v[3 * idx], y = v[3 * idx + 1], z = v[3 * idx + 2];
        double r = 90.0 * (1.0 + 0.12 * sin(3.0 * x + 1.0) * sin(4.0 * y) * cos(2.0 * z + 0.5) + 0.06 * sin(9.0 * x * z));
        out.push_back((float)(r * x));
        out.push_back((float)(r * y + 108.0));
        out.push_back((float)(r * z));
    }
    return out;
}

// tobj 4.0.0 load_obj(triangulate: true) then `models[0]` (src/main.rs:745-789), restated for
// `v` / `f` / `o` / `g` records: vertex positions are global to the file; a model ends
// where an `o` or `g` record follows faces (tobj pushes a Model there and only when it
// has faces), and the reference keeps only the first one; polygons are fan-triangulated
// (v0, v[i-1], v[i]) like tobj's triangulate; indices may be negative (relative) and
// carry /vt/vn parts, which are ignored. Not restated (parity unpinned): tobj splits a
// model at `usemtl` only when an .mtl library defining the material was loaded, and
// emits 1-2 vertex `f` records as points/lines; neither occurs in the reference's meshes.
// True when the line at `i` starts a new tobj model (an `o` or `g` record).
bool model_done(const std::string& text, size_t i) {
    const char c = text[i];
    return (c == 'o' || c == 'g') && i + 1 < text.size() && (text[i + 1] == ' ' || text[i + 1] == '\t');
}

int load_obj_tris(const std::string& path, std::vector<float>* out) {
    std::vector<uint8_t> bytes;
    if (!read_file(path, &bytes)) return set_error(RT_ERR_IO, "cannot read " + path);
    if (bytes.size() < 200 && std::string(bytes.begin(), bytes.end()).find("git-lfs") != std::string::npos)
        return set_error(RT_ERR_IO, path + " is a Git-LFS pointer, not a mesh");
    std::string text(bytes.begin(), bytes.end());
    std::vector<float> pos;
    size_t i = 0;
    while (i < text.size() && !(model_done(text, i) && !out->empty())) {
        size_t e = text.find('\n', i);
        if (e == std::string::npos) e = text.size();
        std::string line = text.substr(i, e - i);
        i = e + 1;
        if (line.size() > 2 && line[0] == 'v' && (line[1] == ' ' || line[1] == '\t')) {
            float x, y, z;
            if (sscanf(line.c_str() + 2, "%f %f %f", &x, &y, &z) == 3) {
                pos.push_back(x);
                pos.push_back(y);
                pos.push_back(z);
            }
        } else if (line.size() > 2 && line[0] == 'f' && (line[1] == ' ' || line[1] == '\t')) {
            std::vector<long> idx;
            const char* p = line.c_str() + 2;
            while (*p) {
                while (*p == ' ' || *p == '\t' || *p == '\r') ++p;
                if (!*p) break;
                long k = strtol(p, (char**)&p, 10);
                while (*p && *p != ' ' && *p != '\t') ++p;
                long nv = (long)(pos.size() / 3);
                long r = k < 0 ? nv + k : k - 1;
                if (r < 0 || r >= nv) return set_error(RT_ERR_INVALID, "OBJ face index out of range in " + path);
                idx.push_back(r);
            }
            for (size_t t = 1; t + 1 < idx.size(); ++t) {
                long tri[3] = {idx[0], idx[t], idx[t + 1]};
                for (long q : tri)
                    for (int c = 0; c < 3; ++c) out->push_back(pos[3 * q + c]);
            }
        }
    }
    if (out->empty()) return set_error(RT_ERR_INVALID, "no triangles in " + path);
    return RT_OK;
}

// src/main.rs:791-829 (bunny / gargoyle / igea_hrpp)
int mesh_scene(SceneBuilder& b, SceneRng& rng, const std::string& dir, const char* file, Vec3 disp, bool synthetic_ok,
               bool predictor,
               int* world) {
    HittableList w = cornell_boundaries(b);
    int white = b.lambertian_from_color(vec3(0.73f, 0.73f, 0.73f));
    std::vector<float> tris;
    std::string path = dir + "/" + file;
    int rc = load_obj_tris(path, &tris);
    if (rc) {
        if (!synthetic_ok) return rc;
        clear_error();
        tris = synthetic_mesh(5);
    }
    HittableList mesh;
    for (size_t i = 0; i + 8 < tris.size(); i += 9)
        mesh.add(b.tri(vec3(tris[i], tris[i + 1], tris[i + 2]), vec3(tris[i + 3], tris[i + 4], tris[i + 5]),
                       vec3(tris[i + 6], tris[i + 7], tris[i + 8]), white));
    int bvh = b.bvh(mesh, 0.0f, 1.0f, rng.next_u64(), predictor);  // igea: Bvh::with_predictor, main.rs:824
    w.add(b.translate(bvh, disp));
    *world = b.list(w);
    return RT_OK;
}

}  // namespace

int generate_scene(const std::string& name, uint64_t seed, const std::string& asset_dir, rt_scene_desc** out) {
    SceneBuilder b;
    SceneRng rng(seed);
    int world = -1, rc;
    if (name == "random-spheres") rc = random_spheres(b, rng, false, true, &world);
    else if (name == "random-spheres-nobvh") rc = random_spheres(b, rng, false, false, &world);
    else if (name == "random-moving-spheres") rc = random_spheres(b, rng, true, true, &world);
    else if (name == "two-spheres") rc = two_spheres(b, &world);
    else if (name == "marble") rc = two_marble_spheres(b, rng, &world);
    else if (name == "earth") rc = earth(b, asset_dir, &world);
    else if (name == "simple-lights") rc = simple_lights(b, rng, &world);
    else if (name == "cornell") rc = cornell(b, false, &world);
    else if (name == "cornell-smoke") rc = cornell(b, true, &world);
    else if (name == "showcase") rc = showcase(b, rng, asset_dir, &world);
    else if (name == "bunny") rc = mesh_scene(b, rng, asset_dir, "bunny_2000_scale.obj", vec3(325.0f, 0.0f, 200.0f), true, false, &world);
    else if (name == "gargoyle") rc = mesh_scene(b, rng, asset_dir, "gargoyle.obj", vec3(275.0f, 0.0f, 200.0f), false, false, &world);
    else if (name == "igea-hrpp") rc = mesh_scene(b, rng, asset_dir, "igea.obj", vec3(275.0f, 0.0f, 200.0f), false, true, &world);
    else return set_error(RT_ERR_INVALID, "unknown scene '" + name + "'");
    if (rc) return rc;
    *out = b.finish(world);
    return RT_OK;
}

int scene_background(const std::string& name, float rgb[3]) {  // src/main.rs:155-164
    static const char* black[] = {"simple-lights", "cornell", "cornell-smoke", "showcase", "bunny", "gargoyle", "igea-hrpp"};
    static const char* sky[] = {"random-spheres", "random-spheres-nobvh", "random-moving-spheres", "two-spheres",
                                "marble", "earth"};
    for (const char* n : black)
        if (name == n) {
            rgb[0] = rgb[1] = rgb[2] = 0.0f;
            return RT_OK;
        }
    for (const char* n : sky)
        if (name == n) {
            rgb[0] = 0.70f;
            rgb[1] = 0.80f;
            rgb[2] = 1.00f;
            return RT_OK;
        }
    return set_error(RT_ERR_INVALID, "unknown scene '" + name + "'");
}

}  // namespace rthost
