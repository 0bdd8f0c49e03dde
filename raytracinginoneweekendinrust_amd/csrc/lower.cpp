// lower.cpp — scene IR -> device SoA layout (see device_scene.hpp).
//
// Host-side construction work the reference does in its constructors:
//   Bvh::new / BvhNode::new_helper   src/bvh.rs:46-62, 249-333 (random split axis,
//                                    stable sort on bounding_box(0,0).min[axis],
//                                    median split, 1- and 2-object leaves)
//   Hittable::bounding_box           per primitive file, cited below
//   Cube::new                        src/geometry/cube.rs:23-81 (six rects, fixed order)
//   RotateY::new                     src/geometry/instance.rs:63-67 (sin / cos)
//   ConstantMedium::new              src/hittable.rs:150-174 (-1 / density)
//   Metal::new                       src/materials/metal.rs:17-22 (fuzz clamp)
//   Perlin::new                      noise 0.8.2 PermutationTable (marble.rs:14)
//   Camera::new                      src/camera.rs:44-81
#include "lower.hpp"

#include <string.h>

#include <algorithm>
#include <cmath>
#include <functional>
#include <unordered_map>

#include "../../include/rt_numeric_spec.h"

namespace rthost {

using rtdev::f4;

uint64_t HostScene::bytes() const {
    return entries.size() * sizeof(rtdev::DevEntry) + sph.size() * 16 + sph_mat.size() * 4 +
           msph.size() * 16 + rect.size() * 16 + tri.size() * 16 + nodes.size() * 16 + nodes2.size() * 16 +
           mats.size() * sizeof(rtdev::DevMaterial) + texs.size() * sizeof(rtdev::DevTexture) +
           perm.size() + texels.size() + hrpp_keys.size() * 8 + hrpp_vals.size() * 4;
}

// ---------------------------------------------------------------------------
// small f32 vector helpers (glam 0.22 evaluation order)
// ---------------------------------------------------------------------------
namespace {
struct V {
    float x, y, z;
};
inline V vadd(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V vsub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V vscale(float s, V a) { return {s * a.x, s * a.y, s * a.z}; }
inline V vdivs(V a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline float vdot(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline V vcross(V a, V b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
inline V vnorm(V a) {
    float r = 1.0f / __builtin_sqrtf(vdot(a, a));
    return {a.x * r, a.y * r, a.z * r};
}
inline float rs_min(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return a < b ? a : b;
}
inline float rs_max(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return a > b ? a : b;
}
inline float rs_clamp(float x, float lo, float hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
struct Box {
    V mn, mx;
};
inline Box box_union(const Box& a, const Box& b) {  // aabb.rs:43-62
    return {{rs_min(a.mn.x, b.mn.x), rs_min(a.mn.y, b.mn.y), rs_min(a.mn.z, b.mn.z)},
            {rs_max(a.mx.x, b.mx.x), rs_max(a.mx.y, b.mx.y), rs_max(a.mx.z, b.mx.z)}};
}
inline int total_cmp(float a, float b) {  // f32::total_cmp
    int32_t l = (int32_t)rt_spec_f32_bits(a), r = (int32_t)rt_spec_f32_bits(b);
    l ^= (int32_t)(((uint32_t)(l >> 31)) >> 1);
    r ^= (int32_t)(((uint32_t)(r >> 31)) >> 1);
    return (l > r) - (l < r);
}
constexpr float kEps = 1.1920929e-07f;  // f32::EPSILON
constexpr float kInfF = __builtin_inff();

inline uint32_t fbits(float f) { return rt_spec_f32_bits(f); }
inline float bitsf(uint32_t u) { return rt_spec_bits_f32(u); }
}  // namespace

// ---------------------------------------------------------------------------
// random streams shared with the oracle
// ---------------------------------------------------------------------------
void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

namespace {
// Split-axis stream of one Bvh::new: Philox key = IR seed, counter (block, 0, 0, 0);
// rand 0.8.5 UniformInt::sample_single_inclusive(0, 2) (bvh.rs:255).
struct AxisStream {
    uint32_t key[2], block = 0, buf[4];
    int idx = 4;
    explicit AxisStream(uint64_t seed) {
        key[0] = (uint32_t)seed;
        key[1] = (uint32_t)(seed >> 32);
    }
    uint32_t next() {
        if (idx == 4) {
            uint32_t ctr[4] = {block++, 0u, 0u, 0u};
            philox4x32_10(ctr, key, buf);
            idx = 0;
        }
        return buf[idx++];
    }
    int axis() {
        const uint32_t range = 3u, zone = (3u << 30) - 1u;
        for (;;) {
            uint64_t m = (uint64_t)next() * range;
            if ((uint32_t)m <= zone) return (int)(m >> 32);
        }
    }
};
}  // namespace

void perlin_permutation(uint32_t seed, uint8_t out[256]) {
    uint32_t x = 1u, y = seed, z = seed, w = seed;  // XorShiftRng::from_seed([1, seed, seed, seed])
    auto next = [&]() {
        uint32_t t = x ^ (x << 11);
        x = y; y = z; z = w;
        w = w ^ (w >> 19) ^ (t ^ (t >> 8));
        return w;
    };
    for (int i = 0; i < 256; ++i) out[i] = (uint8_t)i;
    for (uint32_t i = 255; i >= 1; --i) {  // SliceRandom::shuffle (rand 0.7)
        uint32_t n = i + 1, zone = (n << __builtin_clz(n)) - 1u, j;
        for (;;) {
            uint64_t m = (uint64_t)next() * n;
            if ((uint32_t)m <= zone) {
                j = (uint32_t)(m >> 32);
                break;
            }
        }
        std::swap(out[i], out[j]);
    }
}

// ---------------------------------------------------------------------------
// Camera::new
// ---------------------------------------------------------------------------
int camera_new(const rt_camera_desc* d, rt_camera* c, std::string* err) {
    V lf{d->look_from[0], d->look_from[1], d->look_from[2]};
    V la{d->look_at[0], d->look_at[1], d->look_at[2]};
    V vup{d->view_up[0], d->view_up[1], d->view_up[2]};
    float theta = rt_to_radians(d->vfov_deg);
    float h = rt_tanf(theta / 2.0f);
    float vh = 2.0f * h;
    float vw = d->aspect_ratio * vh;
    V w = vnorm(vsub(lf, la));
    V u = vnorm(vcross(vup, w));
    V v = vcross(w, u);
    V hor = vscale(d->focus_dist * vw, u);
    V ver = vscale(d->focus_dist * vh, v);
    V llc = vsub(vsub(vsub(lf, vdivs(hor, 2.0f)), vdivs(ver, 2.0f)), vscale(d->focus_dist, w));
    auto put = [](float* dst, V a) {
        dst[0] = a.x;
        dst[1] = a.y;
        dst[2] = a.z;
    };
    put(c->origin, lf);
    put(c->horizontal, hor);
    put(c->vertical, ver);
    put(c->lower_left_corner, llc);
    put(c->u, u);
    put(c->v, v);
    c->lens_radius = d->aperture / 2.0f;
    c->time_start = d->time0;
    c->time_end = d->time1;
    if (!(d->time0 <= d->time1)) {
        *err = "Uniform::new_inclusive called with `low > high` (cam time0 > time1)";
        return RT_ERR_INVALID;
    }
    return RT_OK;
}

int camera_device(const rt_camera* c, rtdev::DevCamera* out, std::string* err) {
    memcpy(out->origin, c->origin, sizeof out->origin);
    memcpy(out->horizontal, c->horizontal, sizeof out->horizontal);
    memcpy(out->vertical, c->vertical, sizeof out->vertical);
    memcpy(out->llc, c->lower_left_corner, sizeof out->llc);
    memcpy(out->u, c->u, sizeof out->u);
    memcpy(out->v, c->v, sizeof out->v);
    out->lens_radius = c->lens_radius;
    out->time_low = c->time_start;
    // UniformFloat::new_inclusive (rand 0.8.5) for gen_range(time_start..=time_end), camera.rs:104
    if (!(c->time_start <= c->time_end)) {
        *err = "Uniform::new_inclusive called with `low > high` (camera time_start > time_end)";
        return RT_ERR_INVALID;
    }
    const float max_rand = bitsf(0x3fffffffu | 0x3f800000u) - 1.0f;  // (u32::MAX >> 9) in [1,2) - 1
    float scale = (c->time_end - c->time_start) / max_rand;
    while (scale * max_rand + c->time_start > c->time_end) scale = bitsf(fbits(scale) - 1u);
    out->time_scale = scale;
    return RT_OK;
}

int camera_basis(const rt_camera_desc* d, rtdev::DevCamera* c, std::string* err) {
    rt_camera cam;
    int rc = camera_new(d, &cam, err);
    if (rc) return rc;
    return camera_device(&cam, c, err);
}

// ---------------------------------------------------------------------------
// lowering
// ---------------------------------------------------------------------------
namespace {

struct LeafInfo {
    uint32_t code;
    Box box01;  // bounding_box(time0, time1) of the BVH
    float key[3];
};

class Lowerer {
   public:
    Lowerer(const rt_scene_desc* d, HostScene* out, std::string* err, const BvhOrderer* orderer, int bvh_shape)
        : d_(d), s_(out), err_(err), orderer_(orderer), bvh_shape_(bvh_shape) {}

    int run() {
        if (!d_ || !d_->nodes || d_->num_nodes == 0) return fail(RT_ERR_INVALID, "empty scene");
        if (d_->num_list_items && !d_->list_items) return fail(RT_ERR_INVALID, "list_items is NULL");
        if (d_->world < 0 || (uint32_t)d_->world >= d_->num_nodes || d_->nodes[d_->world].kind != RT_OBJ_LIST)
            return fail(RT_ERR_INVALID, "world must be a LIST node");
        std::vector<rtdev::DevEntry> top;
        Chain chain;
        int rc = lower_entry(d_->world, chain, &top, 0);
        if (rc) return rc;
        // Consecutive untransformed spheres with consecutive records become one
        // run entry (hittable.rs:100-118 order and closest_so_far unchanged): the
        // device then streams the sphere records without per-entry headers.
        // Rectangles the same way (kEntRectRun): a Cornell box's walls and light.
        std::vector<rtdev::DevEntry> merged;
        for (const auto& e : top) {
            const bool rect = e.kind == rtdev::kEntGeom && e.ntf == 0 && rtdev::leaf_type(e.payload) == rtdev::kLeafRect;
            if (rect && !merged.empty()) {
                rtdev::DevEntry& b = merged.back();
                const bool brect = b.kind == rtdev::kEntGeom && b.ntf == 0 && rtdev::leaf_type(b.payload) == rtdev::kLeafRect;
                const uint32_t bfirst = b.kind == rtdev::kEntRectRun ? b.payload : rtdev::leaf_index(b.payload);
                const uint32_t bn = b.kind == rtdev::kEntRectRun ? b.pad[0] : 1u;
                if ((b.kind == rtdev::kEntRectRun || brect) && bfirst + bn == rtdev::leaf_index(e.payload)) {
                    b.kind = rtdev::kEntRectRun;
                    b.payload = bfirst;
                    b.pad[0] = bn + 1u;
                    continue;
                }
            }
            const bool sph = e.kind == rtdev::kEntGeom && e.ntf == 0 &&
                             rtdev::leaf_type(e.payload) == rtdev::kLeafSphere;
            if (sph && !merged.empty()) {
                rtdev::DevEntry& b = merged.back();
                const bool bsph = b.kind == rtdev::kEntGeom && b.ntf == 0 &&
                                  rtdev::leaf_type(b.payload) == rtdev::kLeafSphere;
                const uint32_t bfirst = rtdev::leaf_index(b.payload), bn = b.kind == rtdev::kEntSphereRun ? b.pad[0] : 1u;
                if ((b.kind == rtdev::kEntSphereRun || bsph) && (b.kind == rtdev::kEntSphereRun ? b.payload : bfirst) + bn ==
                                                                   rtdev::leaf_index(e.payload)) {
                    if (b.kind != rtdev::kEntSphereRun) {
                        b.kind = rtdev::kEntSphereRun;
                        b.payload = bfirst;
                    }
                    b.pad[0] = bn + 1u;
                    continue;
                }
            }
            merged.push_back(e);
        }
        top.swap(merged);
        s_->num_top = (uint32_t)top.size();
        for (auto& e : top)
            if (e.kind == rtdev::kEntMedium) e.payload += s_->num_top;
        s_->entries = top;
        s_->entries.insert(s_->entries.end(), aux_.begin(), aux_.end());
        if (s_->entries.empty()) {
            // An empty world: keep one inert entry so device pointers are valid.
            s_->num_top = 0;
        }
        return RT_OK;
    }

   private:
    struct Chain {
        int n = 0;
        f4 op[rtdev::kMaxTransforms];
    };

    int fail(int code, const std::string& m) {
        *err_ = m;
        return code;
    }
    const rt_node& node(int i) const { return d_->nodes[i]; }
    bool valid(int i) const { return i >= 0 && (uint32_t)i < d_->num_nodes; }
    int list_range(const rt_node& n, uint32_t* first, uint32_t* count) {
        if (n.ref[0] < 0 || n.ref[1] < 0 || (uint64_t)n.ref[0] + (uint64_t)n.ref[1] > d_->num_list_items)
            return fail(RT_ERR_INVALID, "LIST range out of bounds");
        *first = (uint32_t)n.ref[0];
        *count = (uint32_t)n.ref[1];
        return RT_OK;
    }

    // --- textures / materials --------------------------------------------
    int lower_texture(int idx, uint32_t* out, int depth) {
        if (!valid(idx)) return fail(RT_ERR_INVALID, "texture ref out of range");
        if (depth > 64) return fail(RT_ERR_INVALID, "texture graph too deep (cycle?)");
        auto it = tex_memo_.find(idx);
        if (it != tex_memo_.end()) {
            *out = it->second;
            return RT_OK;
        }
        const rt_node& n = node(idx);
        rtdev::DevTexture t;
        memset(&t, 0, sizeof t);
        switch (n.kind) {
            case RT_TEX_SOLID:  // solid_color.rs:21-25
                t.kind = rtdev::kTexSolid;
                t.color[0] = n.f[0]; t.color[1] = n.f[1]; t.color[2] = n.f[2];
                break;
            case RT_TEX_CHECKER: {  // checker.rs:27-37
                uint32_t even, odd;
                int rc = lower_texture(n.ref[0], &even, depth + 1);
                if (rc) return rc;
                if ((rc = lower_texture(n.ref[1], &odd, depth + 1))) return rc;
                t.kind = rtdev::kTexChecker;
                t.a = even;
                t.b = odd;
                t.scale = n.f[0];
                break;
            }
            case RT_TEX_MARBLE: {  // marble.rs:13-20: Perlin(seed) + Turbulence distortion Fbm seeds 0..7
                t.kind = rtdev::kTexMarble;
                t.scale = n.f[0];
                t.a = (uint32_t)(s_->perm.size() / 256);
                uint8_t tab[256];
                perlin_permutation((uint32_t)n.seed, tab);
                s_->perm.insert(s_->perm.end(), tab, tab + 256);
                for (uint32_t sd = 0; sd < 8; ++sd) {
                    perlin_permutation(sd, tab);
                    s_->perm.insert(s_->perm.end(), tab, tab + 256);
                }
                break;
            }
            case RT_TEX_IMAGE: {  // image_texture.rs:13-19 (decoded RGB8 supplied in the IR)
                uint64_t w = (uint32_t)n.ref[0], h = (uint32_t)n.ref[1];
                if (n.ref[0] <= 0 || n.ref[1] <= 0) return fail(RT_ERR_INVALID, "image texture with empty size");
                uint64_t need = w * h * 3u;
                if (!d_->image_data || n.seed + need > d_->image_bytes)
                    return fail(RT_ERR_INVALID, "image texture texels out of bounds");
                t.kind = rtdev::kTexImage;
                t.a = (uint32_t)s_->texels.size();
                t.b = (uint32_t)w;
                t.c = (uint32_t)h;
                if (s_->texels.size() + need > 0xffffffffull) return fail(RT_ERR_UNSUPPORTED, "texel pool > 4 GB");
                s_->texels.insert(s_->texels.end(), d_->image_data + n.seed, d_->image_data + n.seed + need);
                break;
            }
            default:
                return fail(RT_ERR_INVALID, "node " + std::to_string(idx) + " is not a texture");
        }
        uint32_t id = (uint32_t)s_->texs.size();
        s_->texs.push_back(t);
        tex_memo_[idx] = id;
        *out = id;
        return RT_OK;
    }

    int lower_material(int idx, uint32_t* out) {
        if (!valid(idx)) return fail(RT_ERR_INVALID, "material ref out of range");
        auto it = mat_memo_.find(idx);
        if (it != mat_memo_.end()) {
            *out = it->second;
            return RT_OK;
        }
        const rt_node& n = node(idx);
        rtdev::DevMaterial m;
        memset(&m, 0, sizeof m);
        int rc = RT_OK;
        switch (n.kind) {
            case RT_MAT_LAMBERTIAN: m.kind = rtdev::kMatLambertian; rc = lower_texture(n.ref[0], &m.tex, 0); break;
            case RT_MAT_DIFFUSE_LIGHT: m.kind = rtdev::kMatLight; rc = lower_texture(n.ref[0], &m.tex, 0); break;
            case RT_MAT_ISOTROPIC: m.kind = rtdev::kMatIsotropic; rc = lower_texture(n.ref[0], &m.tex, 0); break;
            case RT_MAT_METAL:
                m.kind = rtdev::kMatMetal;
                m.albedo[0] = n.f[0]; m.albedo[1] = n.f[1]; m.albedo[2] = n.f[2];
                m.fuzz = rs_clamp(n.f[3], 0.0f, 1.0f);  // metal.rs:20
                break;
            case RT_MAT_DIELECTRIC: m.kind = rtdev::kMatDielectric; m.ior = n.f[0]; break;
            default:
                return fail(RT_ERR_INVALID, "node " + std::to_string(idx) + " is not a material");
        }
        if (rc) return rc;
        if ((m.kind == rtdev::kMatLambertian || m.kind == rtdev::kMatLight || m.kind == rtdev::kMatIsotropic) &&
            texture_reads_uv(m.tex))
            m.flags |= rtdev::kMatNeedsUV;
        uint32_t id = (uint32_t)s_->mats.size();
        s_->mats.push_back(m);
        mat_memo_[idx] = id;
        *out = id;
        return RT_OK;
    }

    // Only ImageTexture::value reads (u, v) (image_texture.rs:21-52); Checker passes them
    // through to its children, Solid and Marble ignore them.
    bool texture_reads_uv(uint32_t t, int depth = 0) const {
        const rtdev::DevTexture& x = s_->texs[t];
        if (x.kind == rtdev::kTexImage) return true;
        if (x.kind == rtdev::kTexChecker && depth < 64) return texture_reads_uv(x.a, depth + 1) || texture_reads_uv(x.b, depth + 1);
        return false;
    }

    uint32_t phase_material(uint32_t tex) {  // Isotropic::new(texture), hittable.rs:159
        auto it = phase_memo_.find(tex);
        if (it != phase_memo_.end()) return it->second;
        rtdev::DevMaterial m;
        memset(&m, 0, sizeof m);
        m.kind = rtdev::kMatIsotropic;
        m.tex = tex;
        if (texture_reads_uv(tex)) m.flags |= rtdev::kMatNeedsUV;
        uint32_t id = (uint32_t)s_->mats.size();
        s_->mats.push_back(m);
        phase_memo_[tex] = id;
        return id;
    }

    // --- primitives ------------------------------------------------------
    static bool is_prim(uint32_t k) {
        return k == RT_OBJ_SPHERE || k == RT_OBJ_MOVING_SPHERE || k == RT_OBJ_XY_RECT || k == RT_OBJ_XZ_RECT ||
               k == RT_OBJ_YZ_RECT || k == RT_OBJ_CUBE || k == RT_OBJ_TRI;
    }

    uint32_t push_rect(uint32_t axis, float a0, float a1, float b0, float b1, float k, uint32_t mat) {
        uint32_t id = (uint32_t)(s_->rect.size() / 2);
        s_->rect.push_back({k, a0, a1, b0});
        s_->rect.push_back({b1, bitsf(axis), bitsf(mat), 0.0f});
        return id;
    }

    void note_coords(const rt_node& n) {
        float m = 0.0f;
        const float* f = n.f;
        auto upd = [&](float v) {
            v = v < 0.0f ? -v : v;
            if (v > m || v != v) m = v != v ? 3.0e38f : v;
        };
        switch (n.kind) {
            case RT_OBJ_SPHERE: for (int i = 0; i < 3; ++i) upd(std::fabs(f[i]) + std::fabs(f[3])); break;
            case RT_OBJ_MOVING_SPHERE:
                for (int i = 0; i < 6; ++i) upd(std::fabs(f[i]) + std::fabs(f[8]));
                break;
            default: for (int i = 0; i < 9; ++i) upd(f[i]); break;
        }
        if (m > s_->coord_bound) s_->coord_bound = m;
    }

    int lower_prim(int idx, uint32_t* code) {
        note_coords(node(idx));
        auto it = prim_memo_.find(idx);
        if (it != prim_memo_.end()) {
            *code = it->second;
            return RT_OK;
        }
        const rt_node& n = node(idx);
        uint32_t mat;
        int rc = lower_material(n.ref[0], &mat);
        if (rc) return rc;
        const float* f = n.f;
        switch (n.kind) {
            case RT_OBJ_SPHERE: {
                uint32_t id = (uint32_t)s_->sph.size();
                s_->sph.push_back({f[0], f[1], f[2], f[3]});
                s_->sph_mat.push_back(mat);
                *code = rtdev::leaf_code(rtdev::kLeafSphere, id);
                break;
            }
            case RT_OBJ_MOVING_SPHERE: {
                uint32_t id = (uint32_t)(s_->msph.size() / 3);
                s_->msph.push_back({f[0], f[1], f[2], f[8]});
                s_->msph.push_back({f[3] - f[0], f[4] - f[1], f[5] - f[2], f[6]});
                s_->msph.push_back({f[7] - f[6], bitsf(mat), 0.0f, 0.0f});
                *code = rtdev::leaf_code(rtdev::kLeafMSphere, id);
                break;
            }
            case RT_OBJ_XY_RECT: *code = rtdev::leaf_code(rtdev::kLeafRect, push_rect(0, f[0], f[1], f[2], f[3], f[4], mat)); break;
            case RT_OBJ_XZ_RECT: *code = rtdev::leaf_code(rtdev::kLeafRect, push_rect(1, f[0], f[1], f[2], f[3], f[4], mat)); break;
            case RT_OBJ_YZ_RECT: *code = rtdev::leaf_code(rtdev::kLeafRect, push_rect(2, f[0], f[1], f[2], f[3], f[4], mat)); break;
            case RT_OBJ_CUBE: {  // cube.rs:25-74
                float x0 = f[0], y0 = f[1], z0 = f[2], x1 = f[3], y1 = f[4], z1 = f[5];
                uint32_t first = push_rect(0, x0, x1, y0, y1, z0, mat);
                push_rect(0, x0, x1, y0, y1, z1, mat);
                push_rect(1, x0, x1, z0, z1, y0, mat);
                push_rect(1, x0, x1, z0, z1, y1, mat);
                push_rect(2, y0, y1, z0, z1, x0, mat);
                push_rect(2, y0, y1, z0, z1, x1, mat);
                *code = rtdev::leaf_code(rtdev::kLeafCube, first);
                break;
            }
            case RT_OBJ_TRI: {
                uint32_t id = (uint32_t)(s_->tri.size() / 3);
                s_->tri.push_back({f[0], f[1], f[2], bitsf(mat)});
                s_->tri.push_back({f[3] - f[0], f[4] - f[1], f[5] - f[2], 0.0f});
                s_->tri.push_back({f[6] - f[0], f[7] - f[1], f[8] - f[2], 0.0f});
                *code = rtdev::leaf_code(rtdev::kLeafTri, id);
                break;
            }
            default:
                return fail(RT_ERR_INVALID, "not a primitive");
        }
        if (rtdev::leaf_index(*code) > rtdev::kMaxIndex - 8) return fail(RT_ERR_UNSUPPORTED, "too many primitives");
        prim_memo_[idx] = *code;
        return RT_OK;
    }

    // Hittable::bounding_box(t0, t1) of a primitive node.
    Box prim_box(const rt_node& n, float t0, float t1) {
        const float* f = n.f;
        switch (n.kind) {
            case RT_OBJ_SPHERE: {  // sphere.rs:105-109
                V c{f[0], f[1], f[2]}, r{f[3], f[3], f[3]};
                return {vsub(c, r), vadd(c, r)};
            }
            case RT_OBJ_MOVING_SPHERE: {  // moving_sphere.rs:86-93 (end_box.min uses time_0)
                V c0{f[0], f[1], f[2]}, c1{f[3], f[4], f[5]}, r{f[8], f[8], f[8]};
                auto center = [&](float time) { return vadd(c0, vscale((time - f[6]) / (f[7] - f[6]), vsub(c1, c0))); };
                Box sb{vsub(center(t0), r), vadd(center(t0), r)};
                Box eb{vsub(center(t0), r), vadd(center(t1), r)};
                return box_union(sb, eb);
            }
            case RT_OBJ_XY_RECT: return {{f[0], f[2], f[4] - kEps}, {f[1], f[3], f[4] + kEps}};  // rectangle.rs:67-73
            case RT_OBJ_XZ_RECT: return {{f[0], f[4] - kEps, f[2]}, {f[1], f[4] + kEps, f[3]}};  // :129-135
            case RT_OBJ_YZ_RECT: return {{f[4] - kEps, f[0], f[2]}, {f[4] + kEps, f[1], f[3]}};  // :191-197
            case RT_OBJ_CUBE: return {{f[0], f[1], f[2]}, {f[3], f[4], f[5]}};                  // cube.rs:95-97
            default: {                                                                         // triangle.rs:94-107
                return {{rs_min(f[0], rs_min(f[3], f[6])) - kEps, rs_min(f[1], rs_min(f[4], f[7])) - kEps,
                         rs_min(f[2], rs_min(f[5], f[8])) - kEps},
                        {rs_max(f[0], rs_max(f[3], f[6])) + kEps, rs_max(f[1], rs_max(f[4], f[7])) + kEps,
                         rs_max(f[2], rs_max(f[5], f[8])) + kEps}};
            }
        }
    }

    // The box a prebuilt tree's leaf slot keeps for the device's conservative leaf
    // reject (leaf_intervals2_nf; prunable BVHs only). The reference tests only the
    // caller's node boxes (bvh.rs:363-417) and stores no shutter times (bvh.rs:38-43),
    // so nothing here may depend on RT_OBJ_BVH_TREE's f[0] / f[1]: a static primitive's
    // own box (time-independent), and an unbounded box for a moving sphere, whose tree is
    // never pruned (its f32 quadratic has no error bound), so the reject never reads it.
    Box leaf_reject_box(const rt_node& c) {
        if (c.kind == RT_OBJ_MOVING_SPHERE) return {{-kInfF, -kInfF, -kInfF}, {kInfF, kInfF, kInfF}};
        return prim_box(c, 0.0f, 0.0f);
    }

    // --- BVH ---------------------------------------------------------------
    struct TNode {
        uint32_t child[2];  // temp node index or leaf code
        bool is_node[2];
        Box box;
        Box leaf_box[2];    // box of a leaf child (device-side conservative leaf test)
    };

    int bvh_build(const rt_node& n, uint32_t* root_out) {
        uint32_t first, count;
        if (!valid(n.ref[0]) || node(n.ref[0]).kind != RT_OBJ_LIST) return fail(RT_ERR_INVALID, "BVH must reference a LIST");
        int rc = list_range(node(n.ref[0]), &first, &count);
        if (rc) return rc;
        if (count == 0) return fail(RT_ERR_INVALID, "BVH over an empty list");
        std::vector<LeafInfo> items(count);
        bool prunable = true;  // closest-hit pruning is proven safe only for these leaf types
        for (uint32_t i = 0; i < count; ++i) {
            int ni = d_->list_items[first + i];
            if (!valid(ni)) return fail(RT_ERR_INVALID, "list item out of range");
            const rt_node& c = node(ni);
            if (!is_prim(c.kind))
                return fail(RT_ERR_UNSUPPORTED, "device BVH leaves must be Sphere/MovingSphere/Rect/Cube/Tri (node " +
                                                    std::to_string(ni) + " kind " + std::to_string(c.kind) + ")");
            if ((rc = lower_prim(ni, &items[i].code))) return rc;
            if (c.kind == RT_OBJ_MOVING_SPHERE || c.kind == RT_OBJ_TRI) prunable = false;
            if (c.kind == RT_OBJ_MOVING_SPHERE || c.kind == RT_OBJ_XY_RECT || c.kind == RT_OBJ_XZ_RECT ||
                c.kind == RT_OBJ_YZ_RECT)
                s_->bvh_rect_msph = true;
            items[i].box01 = prim_box(c, n.f[0], n.f[1]);
            Box b00 = prim_box(c, 0.0f, 0.0f);  // box_compare uses bounding_box(0.0, 0.0), bvh.rs:421-422
            items[i].key[0] = b00.mn.x;
            items[i].key[1] = b00.mn.y;
            items[i].key[2] = b00.mn.z;
        }
        // Large BVHs: the leaf order comes from the device builder; the recursion
        // below then only shapes the tree (which depends on counts alone) and
        // draws the same axis stream.
        bool presorted = false;
        if (orderer_ && count >= orderer_->min_items) {
            std::vector<float> keys(3u * (size_t)count);
            for (uint32_t i = 0; i < count; ++i)
                for (int k = 0; k < 3; ++k) keys[3u * i + k] = items[i].key[k];
            std::vector<uint32_t> order(count, UINT32_MAX);
            std::string e;
            if ((rc = orderer_->fn(orderer_->ctx, keys.data(), count, n.seed, order.data(), &e))) return fail(rc, e);
            std::vector<LeafInfo> sorted(count);
            std::vector<uint8_t> seen(count, 0);
            for (uint32_t i = 0; i < count; ++i) {
                if (order[i] >= count || seen[order[i]]) return fail(RT_ERR_HIP, "device BVH order is not a permutation");
                seen[order[i]] = 1;
                sorted[i] = items[order[i]];
            }
            items.swap(sorted);
            presorted = true;
        }
        std::vector<TNode> tn;
        tn.reserve(count * 2 + 1);
        AxisStream ax(n.seed);
        std::vector<LeafInfo> tmp(count);
        // BvhNode::new_helper, bvh.rs:249-333; returns the temp node index.
        std::function<uint32_t(LeafInfo*, uint32_t, uint32_t)> helper = [&](LeafInfo* o, uint32_t cnt,
                                                                            uint32_t depth) -> uint32_t {
            if (depth > max_depth_) max_depth_ = depth;
            int axis = ax.axis();
            TNode t;
            t.leaf_box[0] = t.leaf_box[1] = Box{{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}};
            if (cnt == 1) {
                t.child[0] = o[0].code;
                t.is_node[0] = false;
                t.child[1] = rtdev::kChildEmpty;  // same object twice in the reference: tested once here
                t.is_node[1] = false;
                t.box = box_union(o[0].box01, o[0].box01);
                t.leaf_box[0] = o[0].box01;
            } else if (cnt == 2) {
                int a = presorted || total_cmp(o[0].key[axis], o[1].key[axis]) < 0 ? 0 : 1;
                t.child[0] = o[a].code;
                t.child[1] = o[1 - a].code;
                t.is_node[0] = t.is_node[1] = false;
                t.box = box_union(o[a].box01, o[1 - a].box01);
                t.leaf_box[0] = o[a].box01;
                t.leaf_box[1] = o[1 - a].box01;
            } else {
                if (!presorted)
                    std::stable_sort(o, o + cnt, [axis](const LeafInfo& p, const LeafInfo& q) {
                        return total_cmp(p.key[axis], q.key[axis]) < 0;
                    });
                uint32_t mid = cnt / 2;
                uint32_t l = helper(o, mid, depth + 1);
                uint32_t r = helper(o + mid, cnt - mid, depth + 1);
                t.child[0] = l;
                t.child[1] = r;
                t.is_node[0] = t.is_node[1] = true;
                t.box = box_union(tn[l].box, tn[r].box);
            }
            tn.push_back(t);
            return (uint32_t)tn.size() - 1;
        };
        uint32_t troot = helper(items.data(), count, 1);
        return bvh_emit(tn, troot, prunable, n.ref[1] == 1, root_out);
    }

    // RT_OBJ_BVH_TREE: a Bvh the caller has already built (bvh.rs:38-43), lowered
    // as given: its shape, boxes and child order decide the visit set and every
    // DFS-rank tie, exactly as BvhNode::hit (bvh.rs:363-417) walks that array.
    int bvh_tree(const rt_node& n, uint32_t* root_out) {
        if (n.ref[0] < 0 || n.ref[1] <= 0 || !d_->bvh_nodes ||
            (uint64_t)n.ref[0] + (uint64_t)n.ref[1] > d_->num_bvh_nodes)
            return fail(RT_ERR_INVALID, "BVH tree node range out of bounds");
        const uint32_t first = (uint32_t)n.ref[0], cnt = (uint32_t)n.ref[1];
        if (n.ref[2] < 0 || (uint32_t)n.ref[2] >= cnt) return fail(RT_ERR_INVALID, "BVH tree root_index out of range");
        const rt_bvh_node* bn = d_->bvh_nodes + first;
        std::vector<TNode> tn(cnt);
        std::vector<uint8_t> seen(cnt, 0);
        bool prunable = true;
        const Box none{{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}};
        auto inside = [](const Box& c, const Box& p) {
            return p.mn.x <= c.mn.x && p.mn.y <= c.mn.y && p.mn.z <= c.mn.z && c.mx.x <= p.mx.x && c.mx.y <= p.mx.y &&
                   c.mx.z <= p.mx.z;
        };
        // iterative preorder walk from the root: every node reached exactly once
        std::vector<std::pair<uint32_t, uint32_t>> st{{(uint32_t)n.ref[2], 1u}};
        while (!st.empty()) {
            const uint32_t i = st.back().first, depth = st.back().second;
            st.pop_back();
            if (seen[i]) return fail(RT_ERR_INVALID, "BVH tree node " + std::to_string(i) + " reached twice");
            seen[i] = 1;
            if (depth > max_depth_) max_depth_ = depth;
            if (depth > 4096) return fail(RT_ERR_UNSUPPORTED, "BVH tree deeper than 4096 levels");
            const rt_bvh_node& b = bn[i];
            TNode& t = tn[i];
            t.box = Box{{b.bbox_min[0], b.bbox_min[1], b.bbox_min[2]}, {b.bbox_max[0], b.bbox_max[1], b.bbox_max[2]}};
            t.leaf_box[0] = t.leaf_box[1] = none;
            const bool lh = (b.flags & RT_BVH_LEFT_HITTABLE) != 0u, rh = (b.flags & RT_BVH_RIGHT_HITTABLE) != 0u;
            if (lh != rh)
                return fail(RT_ERR_UNSUPPORTED, "BVH tree node " + std::to_string(i) +
                                                    " mixes Child::Index and Child::Hittable (new_helper never does)");
            if (lh) {  // the 1-2 object leaves of bvh.rs:260-276
                const int obj[2] = {b.left, b.right};
                for (int k = 0; k < 2; ++k) {
                    if (!valid(obj[k])) return fail(RT_ERR_INVALID, "BVH tree leaf object out of range");
                    const rt_node& c = node(obj[k]);
                    if (!is_prim(c.kind))
                        return fail(RT_ERR_UNSUPPORTED, "device BVH leaves must be Sphere/MovingSphere/Rect/Cube/Tri");
                    if (c.kind == RT_OBJ_MOVING_SPHERE || c.kind == RT_OBJ_TRI) prunable = false;
                    if (c.kind == RT_OBJ_MOVING_SPHERE || c.kind == RT_OBJ_XY_RECT || c.kind == RT_OBJ_XZ_RECT ||
                        c.kind == RT_OBJ_YZ_RECT)
                        s_->bvh_rect_msph = true;
                    // Pruning assumes every primitive lies inside the box the caller gave the node
                    // holding it. The reference only tests those boxes (bvh.rs:363-417), so a tree
                    // that breaks this is legal; it is traversed without pruning.
                    if (!inside(prim_box(c, 0.0f, 0.0f), t.box)) prunable = false;
                }
                int rc;
                t.is_node[0] = t.is_node[1] = false;
                if ((rc = lower_prim(obj[0], &t.child[0]))) return rc;
                t.leaf_box[0] = leaf_reject_box(node(obj[0]));
                if (obj[1] == obj[0]) {  // a 1-object node repeats its object: same result tested once
                    t.child[1] = rtdev::kChildEmpty;
                } else {
                    if ((rc = lower_prim(obj[1], &t.child[1]))) return rc;
                    t.leaf_box[1] = leaf_reject_box(node(obj[1]));
                }
            } else {
                const int ch[2] = {b.left, b.right};
                for (int k = 0; k < 2; ++k) {
                    if (ch[k] < 0 || (uint32_t)ch[k] >= cnt) return fail(RT_ERR_INVALID, "BVH tree child index out of range");
                    t.child[k] = (uint32_t)ch[k];
                    t.is_node[k] = true;
                }
                st.push_back({t.child[1], depth + 1});
                st.push_back({t.child[0], depth + 1});
            }
        }
        // The BVH4 collapse skips the box tests of interior nodes it merges away:
        // exact only when every Index child's box lies inside its parent's (the
        // reference builder's boxes are unions, bvh.rs:294-300, so this holds).
        for (uint32_t i = 0; i < cnt; ++i) {
            if (!seen[i]) return fail(RT_ERR_INVALID, "BVH tree node " + std::to_string(i) + " not reachable from the root");
            for (int k = 0; k < 2; ++k)
                if (tn[i].is_node[k] && !inside(tn[tn[i].child[k]].box, tn[i].box))
                    return fail(RT_ERR_UNSUPPORTED, "BVH tree node " + std::to_string(tn[i].child[k]) +
                                                        ": box not inside its parent's (not a union-built tree)");
        }
        return bvh_emit(tn, (uint32_t)n.ref[2], prunable, n.f[2] == 1.0f, root_out);
    }

    // Lays out one reference BVH2 (tn, root troot) for the device: the BVH4 the fast
    // kernel traverses, the BVH2 the reference kernel replays, HRPP side data.
    int bvh_emit(const std::vector<TNode>& tn, uint32_t troot, bool prunable, bool predictor, uint32_t* root_out) {
        // Leaf children carry their DFS ordinal in the reference tree ("rank",
        // cube faces rank + 0..5): the device may visit children in any order
        // and still resolves equal-t ties like the reference's recursion (later
        // in DFS order wins, bvh.rs:406-414).
        std::vector<uint32_t> rank(tn.size() * 2, 0);
        uint32_t ordinal = 0;
        // the leaf codes in DFS order, bit 31 on the left object of a two-object leaf node (the leaf
        // scan of a triangle BVH entered with a NaN t_max, kernel.hip bvh_hit_nan_tmax)
        std::vector<uint32_t> dfs;
        std::function<void(uint32_t)> ranks = [&](uint32_t i) {
            for (int k = 0; k < 2; ++k) {
                if (tn[i].is_node[k]) {
                    ranks(tn[i].child[k]);
                } else if (tn[i].child[k] != rtdev::kChildEmpty) {
                    rank[2 * i + k] = (++ordinal) * 8u;
                    const bool pair_left = k == 0 && !tn[i].is_node[1] && tn[i].child[1] != rtdev::kChildEmpty;
                    dfs.push_back(tn[i].child[k] | (pair_left ? rtdev::kDfsPairLeft : 0u));
                }
            }
        };
        ranks(troot);
        // Collapse the reference BVH2 into 4-wide nodes (rtdev::kBvhWidth). A wide
        // node made from BVH2 node X starts with X's two children and repeatedly
        // replaces the largest child whose own children are both interior nodes
        // by those two children. Exactness ("BVH4 collapse"): a parent
        // box is the min/max of its children's bounds and the slab arithmetic is
        // monotone, so any child box passing the reference's test implies its
        // skipped parent passes too; and a leaf still sits in the wide node made
        // from its own BVH2 parent, whose box test is exactly the one the
        // reference applies before testing that leaf (bvh.rs:363-417).
        struct Slot {
            bool node;
            uint32_t id;  // temp node index, or leaf code
            Box box;
            uint32_t rank;
        };
        auto area = [](const Box& b) {
            float dx = b.mx.x - b.mn.x, dy = b.mx.y - b.mn.y, dz = b.mx.z - b.mn.z;
            return dx * dy + dy * dz + dz * dx;
        };
        // The binary tree the BVH4 is collapsed from. The reference tree's leaf nodes (the BvhNodes
        // whose children are objects: bvh.rs never mixes objects and nodes under one node) are the
        // units of the fast traversal: a BVH4 leaf node holds one of them and its two objects are
        // tested exactly as BvhNode::hit tests them (bvh.rs:377-414), after the reference's own
        // test of that node's box, which the parent slot holds. Which interior nodes lead there does
        // not change the result: the reference's interior boxes are unions of their children's
        // (bvh.rs:294-300; prebuilt trees are checked for containment), so a leaf node whose own
        // box passes the slab test with the BVH's entry t_max has every reference ancestor pass too
        // (the slab arithmetic is monotone in the box: the BVH4-collapse argument), i.e. it is in
        // the reference's visit set; and an interior node made of unions of leaf-node boxes passes
        // whenever one of its leaf nodes does, so no leaf node of the visit set is ever cut off.
        // Candidates merge by (t, DFS rank) and pruning needs only boxes that contain their
        // objects. So the interior levels are rebuilt here by the surface-area heuristic over the
        // leaf nodes (RT_OPT_BVH_SHAPE 0, the default): the reference's median splits on random axes
        // (bvh.rs:255-257) give boxes that overlap heavily. RT_OPT_BVH_SHAPE 1 collapses the
        // reference tree as built (rounds 1-5). The reference kernel's BVH2 (nodes2) and the DFS
        // ranks always come from the reference tree.
        std::vector<TNode> sah_nodes;  // tn's nodes, then the SAH interior nodes
        const std::vector<TNode>* T = &tn;
        uint32_t root2 = troot;
        if (bvh_shape_ == kBvhShapeSah) {
            std::vector<uint32_t> units;
            std::vector<uint32_t> todo{troot};
            while (!todo.empty()) {
                const uint32_t i = todo.back();
                todo.pop_back();
                if (tn[i].is_node[0] || tn[i].is_node[1]) {
                    for (int k = 0; k < 2; ++k)
                        if (tn[i].is_node[k]) todo.push_back(tn[i].child[k]);
                } else {
                    units.push_back(i);
                }
            }
            if (units.size() >= 3) {
                sah_nodes = tn;
                std::sort(units.begin(), units.end());  // a deterministic start order
                auto cen = [&](uint32_t u, int a) {
                    const Box& b = tn[u].box;
                    return a == 0 ? b.mn.x + b.mx.x : (a == 1 ? b.mn.y + b.mx.y : b.mn.z + b.mx.z);
                };
                std::vector<float> right_area;
                std::function<uint32_t(uint32_t*, uint32_t, uint32_t)> sah = [&](uint32_t* u, uint32_t n,
                                                                                 uint32_t depth) -> uint32_t {
                    if (n == 1) return u[0];
                    int best_axis = -1;
                    uint32_t best_split = n / 2;
                    double best_cost = 0.0;
                    if (depth < 40) {  // (deeper: median splits, so that the tree depth stays bounded)
                        std::vector<uint32_t> v(u, u + n);
                        right_area.assign(n, 0.0f);
                        for (int a = 0; a < 3; ++a) {
                            std::stable_sort(v.begin(), v.end(), [&](uint32_t p, uint32_t q) { return cen(p, a) < cen(q, a); });
                            Box acc = tn[v[n - 1]].box;
                            for (uint32_t i = n - 1; i >= 1; --i) {
                                acc = box_union(acc, tn[v[i]].box);
                                right_area[i] = area(acc);
                            }
                            acc = tn[v[0]].box;
                            for (uint32_t i = 1; i < n; ++i) {  // left = v[0, i), right = v[i, n)
                                const double c = (double)area(acc) * i + (double)right_area[i] * (n - i);
                                if (best_axis < 0 || c < best_cost) {
                                    best_cost = c;
                                    best_axis = a;
                                    best_split = i;
                                }
                                acc = box_union(acc, tn[v[i]].box);
                            }
                        }
                    }
                    const int a = best_axis < 0 ? 0 : best_axis;
                    std::stable_sort(u, u + n, [&](uint32_t p, uint32_t q) { return cen(p, a) < cen(q, a); });
                    const uint32_t l = sah(u, best_split, depth + 1);
                    const uint32_t r = sah(u + best_split, n - best_split, depth + 1);
                    TNode t;
                    t.child[0] = l;
                    t.child[1] = r;
                    t.is_node[0] = t.is_node[1] = true;
                    t.box = box_union(sah_nodes[l].box, sah_nodes[r].box);
                    t.leaf_box[0] = t.leaf_box[1] = Box{{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}};
                    sah_nodes.push_back(t);
                    return (uint32_t)sah_nodes.size() - 1;
                };
                root2 = sah(units.data(), (uint32_t)units.size(), 1);
                T = &sah_nodes;
            }
        }
        const std::vector<TNode>& tt = *T;
        std::vector<std::vector<Slot>> wide;  // per wide node, in DFS preorder
        std::function<uint32_t(uint32_t, uint32_t)> build4 = [&](uint32_t x, uint32_t depth) -> uint32_t {
            std::vector<Slot> sl;
            for (int k = 0; k < 2; ++k) {
                if (tt[x].is_node[k]) sl.push_back({true, tt[x].child[k], tt[tt[x].child[k]].box, 0u});
                else if (tt[x].child[k] != rtdev::kChildEmpty)
                    sl.push_back({false, tt[x].child[k], tt[x].leaf_box[k], rank[2 * x + k]});
            }
            while (sl.size() < rtdev::kBvhWidth) {
                int best = -1;
                for (int k = 0; k < (int)sl.size(); ++k) {
                    if (!sl[k].node) continue;
                    const TNode& c = tt[sl[k].id];
                    if (!(c.is_node[0] && c.is_node[1])) continue;
                    if (best < 0 || area(sl[k].box) > area(sl[best].box)) best = k;
                }
                if (best < 0) break;
                const TNode c = tt[sl[best].id];
                sl[best] = {true, c.child[0], tt[c.child[0]].box, 0u};
                sl.insert(sl.begin() + best + 1, Slot{true, c.child[1], tt[c.child[1]].box, 0u});
            }
            uint32_t me = (uint32_t)wide.size();
            wide.push_back({});
            for (Slot& c : sl)
                if (c.node) c.id = build4(c.id, depth + 1) | 0x40000000u;  // mark: wide index (remapped below)
            wide[me] = sl;
            return me;
        };
        uint32_t wroot = build4(root2, 1);
        // The reference tree itself, as 64 B BVH2 nodes (both children's boxes,
        // child codes), DFS preorder behind a wrapper whose child 0 is the root:
        // traversed in the reference's own recursion order by rays that can take
        // a NaN hit, and by every ray under RT_FLAG_EXACT_BVH (bvh_hit_reference).
        const uint32_t base2 = (uint32_t)(s_->nodes2.size() / 4);
        std::vector<uint32_t> remap2(tn.size());
        uint32_t next2 = base2 + 1;
        std::function<void(uint32_t)> order2 = [&](uint32_t i) {
            remap2[i] = next2++;
            for (int k = 0; k < 2; ++k)
                if (tn[i].is_node[k]) order2(tn[i].child[k]);
        };
        order2(troot);
        if (next2 > rtdev::kMaxIndex) return fail(RT_ERR_UNSUPPORTED, "too many BVH nodes");
        s_->nodes2.resize((size_t)next2 * 4);
        auto put2 = [&](uint32_t o, const Box& lb, const Box& rb, uint32_t lc, uint32_t rc) {
            s_->nodes2[4 * (size_t)o + 0] = {lb.mn.x, lb.mn.y, lb.mn.z, lb.mx.x};
            s_->nodes2[4 * (size_t)o + 1] = {lb.mx.y, lb.mx.z, rb.mn.x, rb.mn.y};
            s_->nodes2[4 * (size_t)o + 2] = {rb.mn.z, rb.mx.x, rb.mx.y, rb.mx.z};
            s_->nodes2[4 * (size_t)o + 3] = {bitsf(lc), bitsf(rc), 0.0f, 0.0f};
        };
        const Box none2{{0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}};
        put2(base2, tn[troot].box, none2, remap2[troot], rtdev::kChildEmpty);
        bool tri_only = true;
        for (const TNode& t : tn)
            for (int k = 0; k < 2; ++k)
                if (!t.is_node[k] && t.child[k] != rtdev::kChildEmpty && rtdev::leaf_type(t.child[k]) != rtdev::kLeafTri)
                    tri_only = false;
        s_->nodes2[4 * (size_t)base2 + 3].w = bitsf(tri_only ? rtdev::kBvh2TriOnly : 0u);
        for (uint32_t i = 0; i < tn.size(); ++i) {
            Box cb[2];
            uint32_t cc[2];
            for (int k = 0; k < 2; ++k) {
                cb[k] = tn[i].is_node[k] ? tn[tn[i].child[k]].box : none2;
                cc[k] = tn[i].is_node[k] ? remap2[tn[i].child[k]] : tn[i].child[k];
            }
            put2(remap2[i], cb[0], cb[1], cc[0], cc[1]);
        }
        uint32_t base = (uint32_t)(s_->nodes.size() / rtdev::kBvhNodeF4);
        uint32_t total = base + 1 + (uint32_t)wide.size();
        if (total >= (rtdev::kLeafNodeFlag >> 1)) return fail(RT_ERR_UNSUPPORTED, "too many BVH nodes");
        s_->nodes.resize((size_t)total * rtdev::kBvhNodeF4);
        auto leaf_node = [&](uint32_t w) {
            for (const Slot& c : wide[w])
                if (c.node) return false;
            return true;
        };
        bool cube_box_mismatch = false;  // (never: put's cube leaves read their leaf box as the cube)
        auto put = [&](uint32_t o, const std::vector<Slot>& sl, uint32_t flags) {
            float mnx[4], mny[4], mnz[4], mxx[4], mxy[4], mxz[4];
            uint32_t ch[4], rk[4];
            for (uint32_t k = 0; k < 4; ++k) {
                const bool have = k < sl.size();
                // an empty slot holds an inverted infinite box: its slab interval is
                // empty for every finite ray (the device's child_keys4 needs no check)
                const Box b = have ? sl[k].box : Box{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
                mnx[k] = b.mn.x; mny[k] = b.mn.y; mnz[k] = b.mn.z;
                mxx[k] = b.mx.x; mxy[k] = b.mx.y; mxz[k] = b.mx.z;
                if (!have) {
                    ch[k] = rtdev::kChildEmpty;
                } else if (sl[k].node) {
                    const uint32_t w = sl[k].id & ~0x40000000u;
                    ch[k] = (base + 1 + w) | (leaf_node(w) ? rtdev::kLeafNodeFlag : 0u);
                } else {
                    ch[k] = sl[k].id;
                }
                rk[k] = have ? sl[k].rank : 0u;
            }
            rk[3] |= flags;
            rtdev::f4* n = &s_->nodes[(size_t)o * rtdev::kBvhNodeF4];
            n[0] = {mnx[0], mnx[1], mnx[2], mnx[3]};
            n[1] = {mny[0], mny[1], mny[2], mny[3]};
            n[2] = {mnz[0], mnz[1], mnz[2], mnz[3]};
            n[3] = {mxx[0], mxx[1], mxx[2], mxx[3]};
            n[4] = {mxy[0], mxy[1], mxy[2], mxy[3]};
            n[5] = {mxz[0], mxz[1], mxz[2], mxz[3]};
            n[6] = {bitsf(ch[0]), bitsf(ch[1]), bitsf(ch[2]), bitsf(ch[3])};
            n[7] = {bitsf(rk[0]), bitsf(rk[1]), bitsf(rk[2]), bitsf(rk[3])};
            // A leaf node (1-2 object slots) carries its spheres in the lanes of the unused slots
            // 2 / 3: slot k's sphere in component 2 + k of rows 0 (cx), 1 (cy), 2 (cz) and 6
            // (radius), which the leaf test reads from the node's own line (kernel.hip bvh_run,
            // RT_LEAF_EMBED) instead of from sph behind the child row. A cube needs nothing: its
            // leaf box (prim_box, cube.rs:95-97) is exactly its six bounds.
            bool leaf = sl.size() <= 2u;
            for (const Slot& c : sl) leaf = leaf && !c.node;
            for (uint32_t k = 0; leaf && k < sl.size(); ++k) {
                const uint32_t code = sl[k].id, idx = rtdev::leaf_index(code);
                auto lane = [&](int row) -> float& { return k ? n[row].w : n[row].z; };
                if (rtdev::leaf_type(code) == rtdev::kLeafSphere) {
                    const rtdev::f4 s = s_->sph[idx];
                    lane(0) = s.x;
                    lane(1) = s.y;
                    lane(2) = s.z;
                    lane(6) = s.w;
                } else if (rtdev::leaf_type(code) == rtdev::kLeafCube) {
                    const rtdev::f4 s0 = s_->rect[2 * (size_t)idx];
                    const Box& b = sl[k].box;
                    const float y1 = s_->rect[2 * (size_t)idx + 1].x, z1 = s_->rect[2 * (size_t)idx + 5].x;
                    if (fbits(b.mn.x) != fbits(s0.y) || fbits(b.mn.y) != fbits(s0.w) || fbits(b.mn.z) != fbits(s0.x) ||
                        fbits(b.mx.x) != fbits(s0.z) || fbits(b.mx.y) != fbits(y1) || fbits(b.mx.z) != fbits(z1))
                        cube_box_mismatch = true;
                }
            }
        };
        // wrapper: slot 0 = the root (its box is tested on entry, bvh.rs:370);
        // its rank[3] carries the BVH's flags
        put(base, {Slot{true, wroot | 0x40000000u, tn[troot].box, 0u}},
            (prunable ? rtdev::kBvhPrunable : 0u) | (tri_only && !prunable ? rtdev::kBvhTriOnly : 0u));
        s_->nodes[(size_t)base * rtdev::kBvhNodeF4 + 7].z = bitsf(base2);  // wrapper rank[2]: the BVH2 wrapper
        if (predictor) {  // Bvh::with_predictor (bvh.rs:69-80): HRPP side data
            // The predictor table stores, per ray hash, "leaf nodes" (GO_UP_LEVEL = 0,
            // bvh.rs:22: the BvhNode whose child object was hit). Each gets a
            // wrapper-format record (its own box, child 0 = the node) so that
            // nodes[p].hit(...) is bvh_hit_reference from that record, and every
            // leaf code maps to it (cube faces too: a cube hit reports its face).
            const uint32_t pid = ++s_->num_predictors;
            s_->nodes2[4 * (size_t)base2 + 3].z = bitsf(pid);
            for (uint32_t i = 0; i < tn.size(); ++i) {
                if (tn[i].is_node[0] || tn[i].is_node[1]) continue;
                const uint32_t w = (uint32_t)(s_->nodes2.size() / 4);
                if (w > rtdev::kMaxIndex) return fail(RT_ERR_UNSUPPORTED, "too many BVH nodes");
                s_->nodes2.resize(s_->nodes2.size() + 4);
                put2(w, tn[i].box, none2, remap2[i], rtdev::kChildEmpty);
                for (int k = 0; k < 2; ++k) {
                    const uint32_t c = tn[i].child[k];
                    if (c == rtdev::kChildEmpty) continue;
                    s_->hrpp_keys.push_back((uint64_t)base2 << 32 | c);
                    s_->hrpp_vals.push_back(w);
                    if (rtdev::leaf_type(c) == rtdev::kLeafCube)
                        for (uint32_t f = 0; f < 6u; ++f) {
                            s_->hrpp_keys.push_back((uint64_t)base2 << 32 |
                                                    rtdev::leaf_code(rtdev::kLeafRect, rtdev::leaf_index(c) + f));
                            s_->hrpp_vals.push_back(w);
                        }
                }
            }
        }
        for (uint32_t w = 0; w < wide.size(); ++w) put(base + 1 + w, wide[w], 0u);
        if (cube_box_mismatch) return fail(RT_ERR_UNSUPPORTED, "internal: a cube leaf's box is not its bounds");
        // The traversal stack a BVH4 walk needs at most: a visit of an interior node with k children
        // pushes the k - 1 it does not descend into first (2 words each) and descends into the
        // nearest, so need(w) = k - 1 + max need(child); a sibling popped later runs with fewer
        // entries of w beneath it. Wide nodes are in preorder (children after parents). The BVH2
        // recursion (reference kernel) keeps one 4-word frame per level.
        std::vector<uint32_t> need(wide.size(), 0u);
        for (uint32_t w = (uint32_t)wide.size(); w-- > 0;) {
            uint32_t deepest = 0, k = 0;
            for (const Slot& c : wide[w]) {
                ++k;
                if (c.node) deepest = std::max(deepest, need[c.id & ~0x40000000u]);
            }
            need[w] = leaf_node(w) ? 0u : (k - 1u) + deepest;
        }
        s_->max_stack = std::max(s_->max_stack, need.empty() ? 1u : std::max(1u, need[0]));
        s_->max_stack_ref = std::max(s_->max_stack_ref, 2u * (max_depth_ + 2u));
        s_->max_bvh_depth = std::max(s_->max_bvh_depth, max_depth_ + 1);
        if (tri_only && !prunable) {
            // A triangle-only BVH's leaf codes in DFS order behind its nodes (whole 8-row nodes: row 0 .x
            // = the count, then four codes a row), its first node index in the wrapper's rank[1].
            const uint32_t tab = (uint32_t)(s_->nodes.size() / rtdev::kBvhNodeF4);
            const size_t rows = 1 + (dfs.size() + 3) / 4;
            const uint32_t nn = (uint32_t)((rows + rtdev::kBvhNodeF4 - 1) / rtdev::kBvhNodeF4);
            if (tab + nn >= (rtdev::kLeafNodeFlag >> 1)) return fail(RT_ERR_UNSUPPORTED, "too many BVH nodes");
            s_->nodes.resize((size_t)(tab + nn) * rtdev::kBvhNodeF4, rtdev::f4{0.0f, 0.0f, 0.0f, 0.0f});
            rtdev::f4* T = &s_->nodes[(size_t)tab * rtdev::kBvhNodeF4];
            T[0].x = bitsf((uint32_t)dfs.size());
            for (size_t i = 0; i < dfs.size(); ++i) {
                rtdev::f4& row = T[1 + i / 4];
                (i % 4 == 0 ? row.x : i % 4 == 1 ? row.y : i % 4 == 2 ? row.z : row.w) = bitsf(dfs[i]);
            }
            s_->nodes[(size_t)base * rtdev::kBvhNodeF4 + 7].y = bitsf(tab);  // wrapper rank[1]
        }
        *root_out = base;
        return RT_OK;
    }

    // --- entries -----------------------------------------------------------
    int lower_entry(int idx, Chain chain, std::vector<rtdev::DevEntry>* out, int depth) {
        if (!valid(idx)) return fail(RT_ERR_INVALID, "hittable ref out of range");
        if (depth > 256) return fail(RT_ERR_INVALID, "hittable graph too deep (cycle?)");
        const rt_node& n = node(idx);
        rtdev::DevEntry e;
        memset(&e, 0, sizeof e);
        e.ntf = (uint32_t)chain.n;
        for (int i = 0; i < chain.n; ++i) e.tf[i] = chain.op[i];
        int rc;
        switch (n.kind) {
            case RT_OBJ_LIST: {  // hittable.rs:100-118 — flattening keeps order and closest_so_far
                uint32_t first, count;
                if ((rc = list_range(n, &first, &count))) return rc;
                for (uint32_t i = 0; i < count; ++i)
                    if ((rc = lower_entry(d_->list_items[first + i], chain, out, depth + 1))) return rc;
                return RT_OK;
            }
            case RT_OBJ_TRANSLATE:
            case RT_OBJ_ROTATE_Y: {
                if (chain.n == rtdev::kMaxTransforms)
                    return fail(RT_ERR_UNSUPPORTED, "more than 3 nested Translate/RotateY");
                Chain c2 = chain;
                if (n.kind == RT_OBJ_TRANSLATE) {
                    translate_sum_ += std::fabs(n.f[0]) + std::fabs(n.f[1]) + std::fabs(n.f[2]);
                    c2.op[c2.n++] = {n.f[0], n.f[1], n.f[2], 0.0f};
                } else {
                    float radians = rt_to_radians(n.f[0]);  // instance.rs:64-67
                    c2.op[c2.n++] = {rt_sinf(radians), rt_cosf(radians), 0.0f, 1.0f};
                }
                return lower_entry(n.ref[0], c2, out, depth + 1);
            }
            case RT_OBJ_BVH:
            case RT_OBJ_BVH_TREE:
                e.kind = rtdev::kEntBvh;
                if ((rc = n.kind == RT_OBJ_BVH ? bvh_build(n, &e.payload) : bvh_tree(n, &e.payload))) return rc;
                out->push_back(e);
                return RT_OK;
            case RT_OBJ_CONSTANT_MEDIUM: {  // hittable.rs:150-174
                std::vector<rtdev::DevEntry> b;
                Chain none;
                if ((rc = lower_entry(n.ref[0], none, &b, depth + 1))) return rc;
                if (b.size() != 1 || b[0].kind == rtdev::kEntMedium)
                    return fail(RT_ERR_UNSUPPORTED, "ConstantMedium boundary must be one primitive/cube/BVH (optionally "
                                                    "under Translate/RotateY)");
                uint32_t tex;
                if ((rc = lower_texture(n.ref[1], &tex, 0))) return rc;
                e.kind = rtdev::kEntMedium;
                e.payload = (uint32_t)aux_.size();  // fixed up by num_top in run()
                e.phase_mat = phase_material(tex);
                e.neg_inv_density = -1.0f / n.f[0];
                aux_.push_back(b[0]);
                out->push_back(e);
                return RT_OK;
            }
            default:
                if (!is_prim(n.kind)) return fail(RT_ERR_INVALID, "node " + std::to_string(idx) + " is not a hittable");
                e.kind = rtdev::kEntGeom;
                if ((rc = lower_prim(idx, &e.payload))) return rc;
                out->push_back(e);
                return RT_OK;
        }
    }

    const rt_scene_desc* d_;
    HostScene* s_;
    std::string* err_;
    const BvhOrderer* orderer_ = nullptr;
    int bvh_shape_ = kBvhShapeSah;
    std::vector<rtdev::DevEntry> aux_;
    std::unordered_map<int, uint32_t> tex_memo_, mat_memo_, prim_memo_, phase_memo_;
    uint32_t max_depth_ = 0;
    float translate_sum_ = 0.0f;

   public:
    float translate_sum() const { return translate_sum_; }
};

}  // namespace

int lower_scene(const rt_scene_desc* desc, HostScene* out, std::string* err, const BvhOrderer* orderer, int bvh_shape) {
    *out = HostScene();
    Lowerer l(desc, out, err, orderer, bvh_shape);
    int rc = l.run();
    {  // HRPP leaf map sorted by key (binary search on the device)
        std::vector<uint32_t> idx(out->hrpp_keys.size());
        for (uint32_t i = 0; i < idx.size(); ++i) idx[i] = i;
        std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return out->hrpp_keys[a] < out->hrpp_keys[b]; });
        std::vector<uint64_t> k(idx.size());
        std::vector<uint32_t> v(idx.size());
        for (uint32_t i = 0; i < idx.size(); ++i) {
            k[i] = out->hrpp_keys[idx[i]];
            v[i] = out->hrpp_vals[idx[i]];
        }
        out->hrpp_keys.swap(k);
        out->hrpp_vals.swap(v);
    }
    out->coord_bound += l.translate_sum();
    return rc;
}

}  // namespace rthost
