/*
 * oracle.c — CPU parity oracle (TEST INFRASTRUCTURE; see oracle.h).
 *
 * Plain-C restatement of jalberse/RayTracingInOneWeekendInRust's hot path.
 * It deliberately keeps the reference's shape — a graph of hittables walked by
 * recursive `hit` calls that build a HitRecord per candidate — instead of the
 * device's flattened SoA traversal, so that the two implementations share
 * nothing but the scene IR (include/rt.h) and the numeric spec
 * (include/rt_numeric_spec.h).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../include/rt_numeric_spec.h"

/* ------------------------------------------------------------------------- */
/* errors                                                                     */
/* ------------------------------------------------------------------------- */
static __thread char g_err[512];
const char* oracle_last_error(void) { return g_err; }
static int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

/* ------------------------------------------------------------------------- */
/* glam 0.22 scalar Vec3 / DVec3, evaluation order as glam's source           */
/* ------------------------------------------------------------------------- */
typedef struct {
    float x, y, z;
} V3;
static inline V3 v3(float x, float y, float z) {
    V3 r = {x, y, z};
    return r;
}
static inline float vget(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 vscale(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
static inline V3 vdivs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline float vdot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline V3 vcross(V3 a, V3 b) {
    return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline float vlen(V3 a) { return __builtin_sqrtf(vdot(a, a)); }
static inline V3 vnorm(V3 a) {
    float r = 1.0f / vlen(a); /* glam: self * self.length().recip() */
    return v3(a.x * r, a.y * r, a.z * r);
}
/* Rust f32::min / f32::max (minnum/maxnum: a NaN operand yields the other). */
static inline float rs_min(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return a < b ? a : b;
}
static inline float rs_max(float a, float b) {
    if (a != a) return b;
    if (b != b) return a;
    return a > b ? a : b;
}
static inline float rs_clamp(float x, float lo, float hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}

typedef struct {
    V3 o, d;
    float time;
} ORay;
static inline V3 ray_at(const ORay* r, float t) { return vadd(r->o, vscale(t, r->d)); } /* ray.rs:28 */

/* ------------------------------------------------------------------------- */
/* Philox4x32-10 (Salmon et al., SC'11 / Random123), independent restatement  */
/* ------------------------------------------------------------------------- */
void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int round = 0; round < 10; ++round) {
        if (round > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* One stream per (pixel, sample): key = seed, counter = (block, sample, pixel, 0).
 * Replaces rand 0.8.5 thread_rng (ChaCha12, OS-seeded; src/renderer.rs:141). */
typedef struct {
    uint32_t key[2];
    uint32_t ctr[4];
    uint32_t buf[4];
    int idx;
} ORng;
static void rng_init(ORng* r, uint64_t seed, uint32_t pixel, uint32_t sample) {
    r->key[0] = (uint32_t)seed;
    r->key[1] = (uint32_t)(seed >> 32);
    r->ctr[0] = 0; r->ctr[1] = sample; r->ctr[2] = pixel; r->ctr[3] = 0;
    r->idx = 4;
}
static inline uint32_t rng_u32(ORng* r) {
    if (r->idx == 4) {
        oracle_philox4x32_10(r->ctr, r->key, r->buf);
        r->ctr[0]++;
        r->idx = 0;
    }
    return r->buf[r->idx++];
}
/* rand 0.8.5 Standard for f32: (u >> 8) * 2^-24, in [0, 1). */
static inline float rng_std01(ORng* r) {
    const float scale = 1.0f / 16777216.0f;
    return scale * (float)(rng_u32(r) >> 8);
}
static inline float f32_from_1_2(uint32_t u) {
    return rt_spec_bits_f32((u >> 9) | 0x3f800000u); /* into_float_with_exponent(0) */
}
/* rand 0.8.5 UniformFloat::sample_single (gen_range(low..high)). */
static float rng_range(ORng* r, float low, float high) {
    float scale = high - low;
    for (;;) {
        float v01 = f32_from_1_2(rng_u32(r)) - 1.0f;
        float res = v01 * scale + low;
        if (res < high) return res;
        scale = rt_spec_bits_f32(rt_spec_f32_bits(scale) - 1u);
    }
}
/* rand 0.8.5 UniformFloat::new_inclusive (gen_range(low..=high), camera.rs:104). */
static int uniform_inclusive(float low, float high, float* out_scale) {
    if (!(low <= high)) return 0;
    const float max_rand = f32_from_1_2(0xffffffffu) - 1.0f;
    float scale = (high - low) / max_rand;
    while (scale * max_rand + low > high) scale = rt_spec_bits_f32(rt_spec_f32_bits(scale) - 1u);
    *out_scale = scale;
    return 1;
}

/* ------------------------------------------------------------------------- */
/* context: random stream, counters, transcendental choice                    */
/* ------------------------------------------------------------------------- */
typedef struct {
    ORng rng;
    oracle_counters* cnt;
    uint32_t flags;
} OCtx;

static inline float o_sin(uint32_t flags, float x) { return (flags & ORACLE_FLAG_LIBM) ? sinf(x) : rt_sinf(x); }
static inline float o_cos(uint32_t flags, float x) { return (flags & ORACLE_FLAG_LIBM) ? cosf(x) : rt_cosf(x); }
static inline float o_tan(uint32_t flags, float x) { return (flags & ORACLE_FLAG_LIBM) ? tanf(x) : rt_tanf(x); }
static inline float o_acos(uint32_t flags, float x) { return (flags & ORACLE_FLAG_LIBM) ? acosf(x) : rt_acosf(x); }
static inline float o_atan2(uint32_t flags, float y, float x) { return (flags & ORACLE_FLAG_LIBM) ? atan2f(y, x) : rt_atan2f(y, x); }
static inline float o_ln(uint32_t flags, float x) { return (flags & ORACLE_FLAG_LIBM) ? logf(x) : rt_logf(x); }

/* src/materials/utils.rs:6-19 */
static V3 random_in_unit_sphere(OCtx* c) {
    for (;;) {
        float x = rng_range(&c->rng, -1.0f, 1.0f);
        float y = rng_range(&c->rng, -1.0f, 1.0f);
        float z = rng_range(&c->rng, -1.0f, 1.0f);
        V3 v = v3(x, y, z);
        if (vdot(v, v) < 1.0f) return v;
    }
}
/* src/utils.rs:9-17 */
static V3 random_in_unit_disk(OCtx* c) {
    for (;;) {
        float x = rng_range(&c->rng, -1.0f, 1.0f);
        float y = rng_range(&c->rng, -1.0f, 1.0f);
        V3 p = v3(x, y, 0.0f);
        if (vdot(p, p) < 1.0f) return p;
    }
}
/* src/utils.rs:5-7 */
static inline int near_zero(V3 v) {
    const float eps = 1.1920929e-07f; /* f32::EPSILON */
    return fabsf(v.x) < eps && fabsf(v.y) < eps && fabsf(v.z) < eps;
}
/* src/materials/utils.rs:37-39 */
static inline V3 reflect(V3 v, V3 n) { return vsub(v, vscale(2.0f * vdot(v, n), n)); }
/* src/materials/utils.rs:41-46 */
static inline V3 refract(V3 uv, V3 n, float eta) {
    float cos_t = rs_min(vdot(vneg(uv), n), 1.0f);
    V3 r_perp = vscale(eta, vadd(uv, vscale(cos_t, n)));
    V3 r_par = vscale(-__builtin_sqrtf(fabsf(1.0f - vdot(r_perp, r_perp))), n);
    return vadd(r_par, r_perp);
}

/* ------------------------------------------------------------------------- */
/* Perlin + Turbulence: restatement of noise 0.8.2 (un-vendored dependency,   */
/* parity unpinned; structure as published): PermutationTable (XorShift128   */
/* seeded [1, seed, seed, seed], rand 0.7 shuffle), surflet perlin_3d,       */
/* Fbm(6 octaves, lacunarity 2pi/3, persistence 0.5), Turbulence(power 1,    */
/* frequency 1, roughness 6, distort seeds 0/1/2) — src/textures/marble.rs.  */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint8_t p[256];
} OPerm;
typedef struct {
    uint32_t x, y, z, w;
} OXorShift;
static uint32_t xorshift_next(OXorShift* s) {
    uint32_t x = s->x;
    uint32_t t = x ^ (x << 11);
    s->x = s->y; s->y = s->z; s->z = s->w;
    uint32_t w = s->w;
    s->w = w ^ (w >> 19) ^ (t ^ (t >> 8));
    return s->w;
}
/* rand 0.7 UniformInt<u32>::sample_single(0, n): widening multiply + zone. */
static uint32_t xorshift_below(OXorShift* s, uint32_t n) {
    uint32_t zone = (n << __builtin_clz(n)) - 1u;
    for (;;) {
        uint64_t m = (uint64_t)xorshift_next(s) * (uint64_t)n;
        if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
    }
}
static void perm_init(OPerm* t, uint32_t seed) {
    OXorShift s = {1u, seed, seed, seed};
    if (s.x == 0 && s.y == 0 && s.z == 0 && s.w == 0) s.x = s.y = s.z = s.w = 0xBAD5EEDu;
    for (int i = 0; i < 256; ++i) t->p[i] = (uint8_t)i;
    for (uint32_t i = 255; i >= 1; --i) {
        uint32_t j = xorshift_below(&s, i + 1);
        uint8_t tmp = t->p[i];
        t->p[i] = t->p[j];
        t->p[j] = tmp;
    }
}
static inline uint32_t perm_hash(const OPerm* t, int64_t x, int64_t y, int64_t z) {
    uint32_t a = t->p[(uint32_t)(x & 0xff)];
    a = t->p[a ^ (uint32_t)(y & 0xff)];
    return t->p[a ^ (uint32_t)(z & 0xff)];
}
static inline double surflet(uint32_t h, double dx, double dy, double dz) {
    const double D = 0.7071067811865476; /* FRAC_1_SQRT_2 */
    double t = 1.0 - ((dx * dx + dy * dy) + dz * dz) * 2.0;
    if (!(t > 0.0)) return 0.0;
    double gx, gy, gz;
    switch (h % 12u) {
        case 0: gx = D; gy = D; gz = 0.0; break;
        case 1: gx = D; gy = -D; gz = 0.0; break;
        case 2: gx = -D; gy = D; gz = 0.0; break;
        case 3: gx = -D; gy = -D; gz = 0.0; break;
        case 4: gx = D; gy = 0.0; gz = D; break;
        case 5: gx = D; gy = 0.0; gz = -D; break;
        case 6: gx = -D; gy = 0.0; gz = D; break;
        case 7: gx = -D; gy = 0.0; gz = -D; break;
        case 8: gx = 0.0; gy = D; gz = D; break;
        case 9: gx = 0.0; gy = D; gz = -D; break;
        case 10: gx = 0.0; gy = -D; gz = D; break;
        default: gx = 0.0; gy = -D; gz = -D; break;
    }
    double t2 = t * t;
    double t4 = t2 * t2;
    return (2.0 * t2 + t4) * ((dx * gx + dy * gy) + dz * gz);
}
static double perlin3(const OPerm* t, double px, double py, double pz) {
    const double SCALE = 1.1547005383792515;
    double fx = floor(px), fy = floor(py), fz = floor(pz);
    int64_t ix = (int64_t)fx, iy = (int64_t)fy, iz = (int64_t)fz;
    double dx = px - fx, dy = py - fy, dz = pz - fz;
    double ex = dx - 1.0, ey = dy - 1.0, ez = dz - 1.0;
    double f000 = surflet(perm_hash(t, ix, iy, iz), dx, dy, dz);
    double f100 = surflet(perm_hash(t, ix + 1, iy, iz), ex, dy, dz);
    double f010 = surflet(perm_hash(t, ix, iy + 1, iz), dx, ey, dz);
    double f110 = surflet(perm_hash(t, ix + 1, iy + 1, iz), ex, ey, dz);
    double f001 = surflet(perm_hash(t, ix, iy, iz + 1), dx, dy, ez);
    double f101 = surflet(perm_hash(t, ix + 1, iy, iz + 1), ex, dy, ez);
    double f011 = surflet(perm_hash(t, ix, iy + 1, iz + 1), dx, ey, ez);
    double f111 = surflet(perm_hash(t, ix + 1, iy + 1, iz + 1), ex, ey, ez);
    double r = (((((((f000 + f100) + f010) + f110) + f001) + f101) + f011) + f111) * SCALE;
    if (r < -1.0) r = -1.0;
    if (r > 1.0) r = 1.0;
    return r;
}
#define FBM_OCTAVES 6
typedef struct {
    OPerm src;
    OPerm fbm[3][FBM_OCTAVES];
} OTurb;
static void turb_init(OTurb* tb, uint32_t seed) {
    perm_init(&tb->src, seed);
    for (int f = 0; f < 3; ++f)
        for (int o = 0; o < FBM_OCTAVES; ++o) perm_init(&tb->fbm[f][o], (uint32_t)(f + o));
}
static double fbm_get(const OPerm* srcs, double x, double y, double z) {
    const double lacunarity = 3.141592653589793 * 2.0 / 3.0;
    double denom = 0.0, pw = 1.0;
    for (int i = 1; i <= FBM_OCTAVES; ++i) {
        pw = pw * 0.5;
        denom = denom + pw;
    }
    const double scale_factor = 1.0 / denom;
    double result = 0.0, persist = 1.0;
    x = x * 1.0; y = y * 1.0; z = z * 1.0; /* frequency 1 */
    for (int o = 0; o < FBM_OCTAVES; ++o) {
        double signal = perlin3(&srcs[o], x, y, z);
        signal = signal * persist;
        result = result + signal;
        persist = persist * 0.5;
        x = x * lacunarity; y = y * lacunarity; z = z * lacunarity;
    }
    return result * scale_factor;
}
static double turb_get(const OTurb* tb, double px, double py, double pz) {
    const double power = 1.0;
    double x0 = px + 12414.0 / 65536.0, y0 = py + 65124.0 / 65536.0, z0 = pz + 31337.0 / 65536.0;
    double x1 = px + 26519.0 / 65536.0, y1 = py + 18128.0 / 65536.0, z1 = pz + 60493.0 / 65536.0;
    double x2 = px + 53820.0 / 65536.0, y2 = py + 11213.0 / 65536.0, z2 = pz + 44845.0 / 65536.0;
    double xd = px + fbm_get(tb->fbm[0], x0, y0, z0) * power;
    double yd = py + fbm_get(tb->fbm[1], x1, y1, z1) * power;
    double zd = pz + fbm_get(tb->fbm[2], x2, y2, z2) * power;
    return perlin3(&tb->src, xd, yd, zd);
}
double oracle_turbulence(uint32_t seed, const double p[3]) {
    OTurb* tb = (OTurb*)malloc(sizeof(OTurb));
    if (!tb) return 0.0;
    turb_init(tb, seed);
    double v = turb_get(tb, p[0], p[1], p[2]);
    free(tb);
    return v;
}

/* ------------------------------------------------------------------------- */
/* scene objects (mirrors of the reference's trait objects)                   */
/* ------------------------------------------------------------------------- */
typedef struct OTex OTex;
struct OTex {
    uint32_t kind;
    V3 color;
    float scale;
    const OTex *even, *odd;
    OTurb* turb;
    const uint8_t* img;
    uint32_t w, h;
};
typedef struct {
    uint32_t kind;
    const OTex* tex;
    V3 albedo;
    float fuzz, ior;
} OMat;
typedef struct {
    V3 mn, mx;
} OAabb;

typedef struct OHit OHit;
typedef struct {
    int is_index;
    int idx;
    const OHit* obj;
} OChild;
typedef struct {
    OChild left, right;
    OAabb box;
} OBvhNode;
typedef struct {
    OBvhNode* nodes;
    int n, cap;
    int root;
} OBvh;

struct OHit {
    uint32_t kind;
    const OMat* mat;
    float f[12];
    const OHit** items; /* LIST / CUBE sides */
    int nitems;
    OBvh bvh;
    const OHit* child;  /* TRANSLATE / ROTATE_Y / MEDIUM boundary */
    V3 disp;
    float sin_t, cos_t;
    int has_rbox;
    OAabb rbox;
    float neg_inv_density;
    OMat phase;
};

typedef struct {
    V3 p, n;
    float t, u, v;
    int front;
    const OMat* mat;
} ORec;

/* arena: every allocation of a scene is freed with it */
typedef struct OBlock {
    struct OBlock* next;
} OBlock;
typedef struct {
    const rt_scene_desc* d;
    void** built;
    OBlock* blocks;
    const OHit* world;
    uint32_t flags;
} OScene;
static void* arena_alloc(OScene* s, size_t n) {
    OBlock* b = (OBlock*)calloc(1, sizeof(OBlock) + n + 16);
    if (!b) return NULL;
    b->next = s->blocks;
    s->blocks = b;
    return (void*)((char*)b + ((sizeof(OBlock) + 15) & ~(size_t)15));
}
static void scene_free(OScene* s) {
    OBlock* b = s->blocks;
    while (b) {
        OBlock* n = b->next;
        free(b);
        b = n;
    }
    free(s->built);
}

/* ------------------------------------------------------------------------- */
/* Aabb (src/aabb.rs)                                                         */
/* ------------------------------------------------------------------------- */
static inline OAabb aabb(V3 mn, V3 mx) {
    OAabb b = {mn, mx};
    return b;
}
/* aabb.rs:28-41 (Kensler slab test; 1/d recomputed per axis per call) */
static int aabb_hit(const OAabb* b, const ORay* r, float t_min, float t_max) {
    for (int i = 0; i < 3; ++i) {
        float inv_d = 1.0f / vget(r->d, i);
        float t0 = (vget(b->mn, i) - vget(r->o, i)) * inv_d;
        float t1 = (vget(b->mx, i) - vget(r->o, i)) * inv_d;
        if (inv_d < 0.0f) {
            float tmp = t0;
            t0 = t1;
            t1 = tmp;
        }
        t_min = t0 > t_min ? t0 : t_min;
        t_max = t1 < t_max ? t1 : t_max;
        if (t_max < t_min) return 0;
    }
    return 1;
}
/* aabb.rs:43-62 */
static OAabb aabb_union2(OAabb a, OAabb b) {
    return aabb(v3(rs_min(a.mn.x, b.mn.x), rs_min(a.mn.y, b.mn.y), rs_min(a.mn.z, b.mn.z)),
                v3(rs_max(a.mx.x, b.mx.x), rs_max(a.mx.y, b.mx.y), rs_max(a.mx.z, b.mx.z)));
}

int oracle_aabb_hit(const float mn[3], const float mx[3], const float o[3], const float d[3],
                    float tmin, float tmax) {
    OAabb b = aabb(v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2]));
    ORay r = {v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), 0.0f};
    return aabb_hit(&b, &r, tmin, tmax);
}
int oracle_aabb_union(const float* a, const float* b, float out[6]) {
    if (!a && !b) return 0;
    if (!a || !b) {
        const float* s = a ? a : b;
        memcpy(out, s, 6 * sizeof(float));
        return 1;
    }
    OAabb r = aabb_union2(aabb(v3(a[0], a[1], a[2]), v3(a[3], a[4], a[5])),
                          aabb(v3(b[0], b[1], b[2]), v3(b[3], b[4], b[5])));
    out[0] = r.mn.x; out[1] = r.mn.y; out[2] = r.mn.z;
    out[3] = r.mx.x; out[4] = r.mx.y; out[5] = r.mx.z;
    return 1;
}

/* ------------------------------------------------------------------------- */
/* HitRecord (src/hittable.rs:28-61)                                          */
/* ------------------------------------------------------------------------- */
static inline void rec_new(ORec* rec, const ORay* r, V3 outward, float t, float u, float v,
                           const OMat* mat) {
    rec->p = ray_at(r, t);
    rec->front = signbit(vdot(r->d, outward)) != 0; /* is_sign_negative */
    rec->n = rec->front ? outward : vneg(outward);
    rec->t = t;
    rec->u = u;
    rec->v = v;
    rec->mat = mat;
}

/* src/geometry/sphere.rs:41-46 */
static void sphere_uv(uint32_t flags, V3 p, float* u, float* v) {
    const float PI = 3.14159265358979323846f;
    const float TWO_PI = 2.0f * PI;
    float theta = o_acos(flags, -p.y);
    float phi = o_atan2(flags, -p.z, p.x) + PI;
    *u = phi / TWO_PI;
    *v = theta / PI;
}
void oracle_sphere_uv(const float p[3], float uv[2]) { sphere_uv(0, v3(p[0], p[1], p[2]), &uv[0], &uv[1]); }

/* ------------------------------------------------------------------------- */
/* bounding boxes (Hittable::bounding_box)                                    */
/* ------------------------------------------------------------------------- */
static V3 msphere_center(const OHit* h, float time) { /* moving_sphere.rs:47-51 */
    V3 c0 = v3(h->f[0], h->f[1], h->f[2]), c1 = v3(h->f[3], h->f[4], h->f[5]);
    return vadd(c0, vscale((time - h->f[6]) / (h->f[7] - h->f[6]), vsub(c1, c0)));
}
static int bvh_bbox(const OBvh* b, OAabb* out) {
    *out = b->nodes[b->root].box;
    return 1;
}
static int hittable_bbox(const OHit* h, float t0, float t1, OAabb* out) {
    const float EPS = 1.1920929e-07f;
    switch (h->kind) {
        case RT_OBJ_SPHERE: { /* sphere.rs:105-109 */
            V3 c = v3(h->f[0], h->f[1], h->f[2]);
            V3 rad = v3(h->f[3], h->f[3], h->f[3]);
            *out = aabb(vsub(c, rad), vadd(c, rad));
            return 1;
        }
        case RT_OBJ_MOVING_SPHERE: { /* moving_sphere.rs:86-93 (end_box.min uses time_0) */
            V3 rad = v3(h->f[8], h->f[8], h->f[8]);
            OAabb sb = aabb(vsub(msphere_center(h, t0), rad), vadd(msphere_center(h, t0), rad));
            OAabb eb = aabb(vsub(msphere_center(h, t0), rad), vadd(msphere_center(h, t1), rad));
            *out = aabb_union2(sb, eb);
            return 1;
        }
        case RT_OBJ_XY_RECT: /* rectangle.rs:67-73 */
            *out = aabb(v3(h->f[0], h->f[2], h->f[4] - EPS), v3(h->f[1], h->f[3], h->f[4] + EPS));
            return 1;
        case RT_OBJ_XZ_RECT: /* rectangle.rs:129-135 */
            *out = aabb(v3(h->f[0], h->f[4] - EPS, h->f[2]), v3(h->f[1], h->f[4] + EPS, h->f[3]));
            return 1;
        case RT_OBJ_YZ_RECT: /* rectangle.rs:191-197 */
            *out = aabb(v3(h->f[4] - EPS, h->f[0], h->f[2]), v3(h->f[4] + EPS, h->f[1], h->f[3]));
            return 1;
        case RT_OBJ_CUBE: /* cube.rs:95-97 */
            *out = aabb(v3(h->f[0], h->f[1], h->f[2]), v3(h->f[3], h->f[4], h->f[5]));
            return 1;
        case RT_OBJ_TRI: { /* triangle.rs:94-107 */
            float mnx = rs_min(h->f[0], rs_min(h->f[3], h->f[6])) - EPS;
            float mny = rs_min(h->f[1], rs_min(h->f[4], h->f[7])) - EPS;
            float mnz = rs_min(h->f[2], rs_min(h->f[5], h->f[8])) - EPS;
            float mxx = rs_max(h->f[0], rs_max(h->f[3], h->f[6])) + EPS;
            float mxy = rs_max(h->f[1], rs_max(h->f[4], h->f[7])) + EPS;
            float mxz = rs_max(h->f[2], rs_max(h->f[5], h->f[8])) + EPS;
            *out = aabb(v3(mnx, mny, mnz), v3(mxx, mxy, mxz));
            return 1;
        }
        case RT_OBJ_LIST: { /* hittable.rs:123-139 */
            if (h->nitems == 0) return 0;
            int have = 0;
            OAabb acc;
            for (int i = 0; i < h->nitems; ++i) {
                OAabb b;
                if (!hittable_bbox(h->items[i], t0, t1, &b)) return 0;
                acc = have ? aabb_union2(acc, b) : b;
                have = 1;
            }
            *out = acc;
            return 1;
        }
        case RT_OBJ_BVH: /* bvh.rs:102-104 */
        case RT_OBJ_BVH_TREE:
            return bvh_bbox(&h->bvh, out);
        case RT_OBJ_TRANSLATE: { /* instance.rs:45-52 */
            OAabb b;
            if (!hittable_bbox(h->child, t0, t1, &b)) return 0;
            *out = aabb(vadd(b.mn, h->disp), vadd(b.mx, h->disp));
            return 1;
        }
        case RT_OBJ_ROTATE_Y: /* instance.rs:145-147 */
            if (!h->has_rbox) return 0;
            *out = h->rbox;
            return 1;
        case RT_OBJ_CONSTANT_MEDIUM: /* hittable.rs:235-237 */
            return hittable_bbox(h->child, t0, t1, out);
        default:
            return 0;
    }
}

/* ------------------------------------------------------------------------- */
/* BVH construction (src/bvh.rs:46-62, 249-333, 420-440)                      */
/* ------------------------------------------------------------------------- */
/* f32::total_cmp */
static int total_cmp(float a, float b) {
    int32_t l = (int32_t)rt_spec_f32_bits(a), r = (int32_t)rt_spec_f32_bits(b);
    l ^= (int32_t)(((uint32_t)(l >> 31)) >> 1);
    r ^= (int32_t)(((uint32_t)(r >> 31)) >> 1);
    return (l > r) - (l < r);
}
typedef struct {
    const OHit* obj;
    float key[3]; /* bounding_box(0.0, 0.0).min, bvh.rs:420-430 */
} OSortItem;
/* Split-axis stream: Philox keyed by the node's seed; rand 0.8.5
 * UniformInt::sample_single_inclusive(0, 2) (widening multiply + zone). */
typedef struct {
    ORng r;
} OAxisRng;
static int axis_draw(OAxisRng* a) {
    const uint32_t range = 3u, zone = (3u << 30) - 1u;
    for (;;) {
        uint64_t m = (uint64_t)rng_u32(&a->r) * range;
        if ((uint32_t)m <= zone) return (int)(m >> 32);
    }
}
static void merge_sort_axis(OSortItem* a, OSortItem* tmp, int n, int axis) { /* stable */
    if (n < 2) return;
    int mid = n / 2;
    merge_sort_axis(a, tmp, mid, axis);
    merge_sort_axis(a + mid, tmp, n - mid, axis);
    int i = 0, j = mid, k = 0;
    while (i < mid && j < n) {
        if (total_cmp(a[j].key[axis], a[i].key[axis]) < 0) tmp[k++] = a[j++];
        else tmp[k++] = a[i++];
    }
    while (i < mid) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, (size_t)n * sizeof(OSortItem));
}
static int bvh_child_box(const OBvh* b, OChild c, float t0, float t1, OAabb* out) {
    if (c.is_index) {
        *out = b->nodes[c.idx].box;
        return 1;
    }
    return hittable_bbox(c.obj, t0, t1, out);
}
static int bvh_new_helper(OBvh* b, OSortItem* objs, OSortItem* tmp, int n, float t0, float t1,
                          OAxisRng* ar, int* err) {
    int axis = axis_draw(ar);
    OChild left, right;
    memset(&left, 0, sizeof left);
    memset(&right, 0, sizeof right);
    if (n == 1) {
        left.obj = right.obj = objs[0].obj;
    } else if (n == 2) {
        if (total_cmp(objs[0].key[axis], objs[1].key[axis]) < 0) {
            left.obj = objs[0].obj;
            right.obj = objs[1].obj;
        } else {
            left.obj = objs[1].obj;
            right.obj = objs[0].obj;
        }
    } else {
        merge_sort_axis(objs, tmp, n, axis);
        int mid = n / 2;
        left.is_index = 1;
        left.idx = bvh_new_helper(b, objs, tmp, mid, t0, t1, ar, err);
        right.is_index = 1;
        right.idx = bvh_new_helper(b, objs + mid, tmp, n - mid, t0, t1, ar, err);
        if (*err) return -1;
    }
    OAabb lb, rb;
    if (!bvh_child_box(b, left, t0, t1, &lb) || !bvh_child_box(b, right, t0, t1, &rb)) {
        *err = 1; /* "Missing bounding box in BVH construction" */
        return -1;
    }
    if (b->n == b->cap) {
        *err = 2;
        return -1;
    }
    OBvhNode* nd = &b->nodes[b->n];
    nd->left = left;
    nd->right = right;
    nd->box = aabb_union2(lb, rb);
    return b->n++;
}

/* The leaf order bvh_new_helper leaves its items in (bvh.rs:249-333), for the
 * device builder's parity tests: the same axis stream, stable merge sort and
 * two-item comparison, on items identified by index. */
static void bvh_order_helper(OSortItem* objs, OSortItem* tmp, int n, OAxisRng* ar) {
    int axis = axis_draw(ar);
    if (n == 2) {
        if (!(total_cmp(objs[0].key[axis], objs[1].key[axis]) < 0)) {
            OSortItem t = objs[0];
            objs[0] = objs[1];
            objs[1] = t;
        }
    } else if (n > 2) {
        merge_sort_axis(objs, tmp, n, axis);
        int mid = n / 2;
        bvh_order_helper(objs, tmp, mid, ar);
        bvh_order_helper(objs + mid, tmp, n - mid, ar);
    }
}
int oracle_bvh_order(const float* keys, uint32_t n, uint64_t seed, uint32_t* order) {
    if (n == 0) return 0;
    OSortItem* it = (OSortItem*)malloc(2u * (size_t)n * sizeof(OSortItem));
    if (!it) return -4;
    for (uint32_t i = 0; i < n; ++i) {
        it[i].obj = (const OHit*)(uintptr_t)(i + 1u);
        for (int k = 0; k < 3; ++k) it[i].key[k] = keys[3u * i + k];
    }
    OAxisRng ar;
    rng_init(&ar.r, seed, 0u, 0u);
    bvh_order_helper(it, it + n, (int)n, &ar);
    for (uint32_t i = 0; i < n; ++i) order[i] = (uint32_t)((uintptr_t)it[i].obj - 1u);
    free(it);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* building the object graph from the IR                                      */
/* ------------------------------------------------------------------------- */
static int build_node(OScene* s, int idx, void** out);

static int get_tex(OScene* s, int idx, const OTex** out) {
    void* p;
    int rc = build_node(s, idx, &p);
    if (rc) return rc;
    uint32_t k = s->d->nodes[idx].kind;
    if (k < RT_TEX_SOLID || k > RT_TEX_IMAGE) return fail(RT_ERR_INVALID, "node %d is not a texture", idx);
    *out = (const OTex*)p;
    return 0;
}
static int get_mat(OScene* s, int idx, const OMat** out) {
    void* p;
    int rc = build_node(s, idx, &p);
    if (rc) return rc;
    uint32_t k = s->d->nodes[idx].kind;
    if (k < RT_MAT_LAMBERTIAN || k > RT_MAT_ISOTROPIC) return fail(RT_ERR_INVALID, "node %d is not a material", idx);
    *out = (const OMat*)p;
    return 0;
}
static int get_hit(OScene* s, int idx, const OHit** out) {
    void* p;
    int rc = build_node(s, idx, &p);
    if (rc) return rc;
    uint32_t k = s->d->nodes[idx].kind;
    if (k < RT_OBJ_SPHERE || k > RT_OBJ_BVH_TREE) return fail(RT_ERR_INVALID, "node %d is not a hittable", idx);
    *out = (const OHit*)p;
    return 0;
}
static OHit* new_rect(OScene* s, uint32_t kind, float a0, float a1, float b0, float b1, float k,
                      const OMat* m) {
    OHit* h = (OHit*)arena_alloc(s, sizeof(OHit));
    if (!h) return NULL;
    h->kind = kind;
    h->f[0] = a0; h->f[1] = a1; h->f[2] = b0; h->f[3] = b1; h->f[4] = k;
    h->mat = m;
    return h;
}
static int build_list_items(OScene* s, const rt_node* n, const OHit*** items, int* count) {
    int first = n->ref[0], cnt = n->ref[1];
    if (cnt < 0 || first < 0 || (uint64_t)first + (uint64_t)cnt > s->d->num_list_items)
        return fail(RT_ERR_INVALID, "list range out of bounds");
    const OHit** it = (const OHit**)arena_alloc(s, sizeof(OHit*) * (size_t)(cnt > 0 ? cnt : 1));
    if (!it) return fail(RT_ERR_OOM, "oom");
    for (int i = 0; i < cnt; ++i) {
        int rc = get_hit(s, s->d->list_items[first + i], &it[i]);
        if (rc) return rc;
    }
    *items = it;
    *count = cnt;
    return 0;
}

static int build_node(OScene* s, int idx, void** out) {
    if (idx < 0 || (uint32_t)idx >= s->d->num_nodes) return fail(RT_ERR_INVALID, "node ref %d out of range", idx);
    if (s->built[idx]) {
        *out = s->built[idx];
        return 0;
    }
    const rt_node* n = &s->d->nodes[idx];
    int rc;
    switch (n->kind) {
        case RT_TEX_SOLID:
        case RT_TEX_CHECKER:
        case RT_TEX_MARBLE:
        case RT_TEX_IMAGE: {
            OTex* t = (OTex*)arena_alloc(s, sizeof(OTex));
            if (!t) return fail(RT_ERR_OOM, "oom");
            t->kind = n->kind;
            t->color = v3(n->f[0], n->f[1], n->f[2]);
            t->scale = n->f[0];
            if (n->kind == RT_TEX_CHECKER) {
                if ((rc = get_tex(s, n->ref[0], &t->even))) return rc;
                if ((rc = get_tex(s, n->ref[1], &t->odd))) return rc;
            } else if (n->kind == RT_TEX_MARBLE) {
                t->turb = (OTurb*)arena_alloc(s, sizeof(OTurb));
                if (!t->turb) return fail(RT_ERR_OOM, "oom");
                turb_init(t->turb, (uint32_t)n->seed);
            } else if (n->kind == RT_TEX_IMAGE) {
                t->w = (uint32_t)n->ref[0];
                t->h = (uint32_t)n->ref[1];
                uint64_t need = (uint64_t)t->w * t->h * 3u;
                if (t->w == 0 || t->h == 0 || n->seed + need > s->d->image_bytes || !s->d->image_data)
                    return fail(RT_ERR_INVALID, "image texture %d out of bounds", idx);
                t->img = s->d->image_data + n->seed;
            }
            *out = s->built[idx] = t;
            return 0;
        }
        case RT_MAT_LAMBERTIAN:
        case RT_MAT_METAL:
        case RT_MAT_DIELECTRIC:
        case RT_MAT_DIFFUSE_LIGHT:
        case RT_MAT_ISOTROPIC: {
            OMat* m = (OMat*)arena_alloc(s, sizeof(OMat));
            if (!m) return fail(RT_ERR_OOM, "oom");
            m->kind = n->kind;
            if (n->kind == RT_MAT_METAL) {
                m->albedo = v3(n->f[0], n->f[1], n->f[2]);
                m->fuzz = rs_clamp(n->f[3], 0.0f, 1.0f); /* metal.rs:20 */
            } else if (n->kind == RT_MAT_DIELECTRIC) {
                m->ior = n->f[0];
            } else {
                if ((rc = get_tex(s, n->ref[0], &m->tex))) return rc;
            }
            *out = s->built[idx] = m;
            return 0;
        }
        default:
            break;
    }
    if (n->kind < RT_OBJ_SPHERE || n->kind > RT_OBJ_BVH_TREE)
        return fail(RT_ERR_INVALID, "node %d: unknown kind %u", idx, n->kind);
    OHit* h = (OHit*)arena_alloc(s, sizeof(OHit));
    if (!h) return fail(RT_ERR_OOM, "oom");
    h->kind = n->kind;
    memcpy(h->f, n->f, sizeof h->f);
    s->built[idx] = h; /* set early: a DAG may revisit, a cycle would be invalid IR */
    switch (n->kind) {
        case RT_OBJ_SPHERE:
        case RT_OBJ_MOVING_SPHERE:
        case RT_OBJ_XY_RECT:
        case RT_OBJ_XZ_RECT:
        case RT_OBJ_YZ_RECT:
        case RT_OBJ_TRI:
            if ((rc = get_mat(s, n->ref[0], &h->mat))) return rc;
            break;
        case RT_OBJ_CUBE: { /* cube.rs:23-81: six rects, fixed order */
            const OMat* m;
            if ((rc = get_mat(s, n->ref[0], &m))) return rc;
            h->mat = m;
            float x0 = n->f[0], y0 = n->f[1], z0 = n->f[2], x1 = n->f[3], y1 = n->f[4], z1 = n->f[5];
            const OHit** sides = (const OHit**)arena_alloc(s, 6 * sizeof(OHit*));
            if (!sides) return fail(RT_ERR_OOM, "oom");
            sides[0] = new_rect(s, RT_OBJ_XY_RECT, x0, x1, y0, y1, z0, m);
            sides[1] = new_rect(s, RT_OBJ_XY_RECT, x0, x1, y0, y1, z1, m);
            sides[2] = new_rect(s, RT_OBJ_XZ_RECT, x0, x1, z0, z1, y0, m);
            sides[3] = new_rect(s, RT_OBJ_XZ_RECT, x0, x1, z0, z1, y1, m);
            sides[4] = new_rect(s, RT_OBJ_YZ_RECT, y0, y1, z0, z1, x0, m);
            sides[5] = new_rect(s, RT_OBJ_YZ_RECT, y0, y1, z0, z1, x1, m);
            for (int i = 0; i < 6; ++i)
                if (!sides[i]) return fail(RT_ERR_OOM, "oom");
            h->items = sides;
            h->nitems = 6;
            break;
        }
        case RT_OBJ_LIST:
            if ((rc = build_list_items(s, n, &h->items, &h->nitems))) return rc;
            break;
        case RT_OBJ_BVH: { /* bvh.rs:46-62 */
            int li = n->ref[0];
            if (li < 0 || (uint32_t)li >= s->d->num_nodes || s->d->nodes[li].kind != RT_OBJ_LIST)
                return fail(RT_ERR_INVALID, "BVH %d must reference a LIST", idx);
            const OHit** items;
            int cnt;
            if ((rc = build_list_items(s, &s->d->nodes[li], &items, &cnt))) return rc;
            if (cnt == 0) return fail(RT_ERR_INVALID, "BVH %d over an empty list", idx);
            OSortItem* objs = (OSortItem*)malloc(sizeof(OSortItem) * (size_t)cnt * 2);
            if (!objs) return fail(RT_ERR_OOM, "oom");
            for (int i = 0; i < cnt; ++i) {
                OAabb bb;
                if (!hittable_bbox(items[i], 0.0f, 0.0f, &bb)) {
                    free(objs);
                    return fail(RT_ERR_INVALID, "Missing bounding box in Bvh construction!");
                }
                objs[i].obj = items[i];
                objs[i].key[0] = bb.mn.x; objs[i].key[1] = bb.mn.y; objs[i].key[2] = bb.mn.z;
            }
            h->bvh.cap = cnt * 2 + 1;
            h->bvh.nodes = (OBvhNode*)arena_alloc(s, sizeof(OBvhNode) * (size_t)h->bvh.cap);
            if (!h->bvh.nodes) {
                free(objs);
                return fail(RT_ERR_OOM, "oom");
            }
            OAxisRng ar;
            rng_init(&ar.r, n->seed, 0u, 0u);
            int err = 0;
            h->bvh.root = bvh_new_helper(&h->bvh, objs, objs + cnt, cnt, n->f[0], n->f[1], &ar, &err);
            free(objs);
            if (err) return fail(RT_ERR_INVALID, "Missing bounding box in BVH construction");
            break;
        }
        case RT_OBJ_BVH_TREE: { /* an already built Bvh (bvh.rs:38-43): BvhNode array as given */
            const rt_bvh_node* bn = s->d->bvh_nodes;
            if (n->ref[0] < 0 || n->ref[1] <= 0 || !bn ||
                (uint64_t)n->ref[0] + (uint64_t)n->ref[1] > s->d->num_bvh_nodes)
                return fail(RT_ERR_INVALID, "BVH tree %d: node range out of bounds", idx);
            if (n->ref[2] < 0 || n->ref[2] >= n->ref[1]) return fail(RT_ERR_INVALID, "BVH tree %d: bad root", idx);
            int cnt = n->ref[1];
            h->bvh.cap = h->bvh.n = cnt;
            h->bvh.root = n->ref[2];
            h->bvh.nodes = (OBvhNode*)arena_alloc(s, sizeof(OBvhNode) * (size_t)cnt);
            if (!h->bvh.nodes) return fail(RT_ERR_OOM, "oom");
            for (int i = 0; i < cnt; ++i) {
                const rt_bvh_node* b = &bn[n->ref[0] + i];
                OBvhNode* nd = &h->bvh.nodes[i];
                OChild* ch[2] = {&nd->left, &nd->right};
                int32_t ref[2] = {b->left, b->right};
                uint32_t hit_flag[2] = {RT_BVH_LEFT_HITTABLE, RT_BVH_RIGHT_HITTABLE};
                for (int k = 0; k < 2; ++k) {
                    memset(ch[k], 0, sizeof *ch[k]);
                    if (b->flags & hit_flag[k]) { /* Child::Hittable */
                        if ((rc = get_hit(s, ref[k], &ch[k]->obj))) return rc;
                    } else { /* Child::Index */
                        if (ref[k] < 0 || ref[k] >= cnt) return fail(RT_ERR_INVALID, "BVH tree %d: child out of range", idx);
                        ch[k]->is_index = 1;
                        ch[k]->idx = ref[k];
                    }
                }
                nd->box.mn = v3(b->bbox_min[0], b->bbox_min[1], b->bbox_min[2]);
                nd->box.mx = v3(b->bbox_max[0], b->bbox_max[1], b->bbox_max[2]);
            }
            break;
        }
        case RT_OBJ_TRANSLATE:
            if ((rc = get_hit(s, n->ref[0], &h->child))) return rc;
            h->disp = v3(n->f[0], n->f[1], n->f[2]);
            break;
        case RT_OBJ_ROTATE_Y: { /* instance.rs:63-102 (bbox loop folds only x,y) */
            if ((rc = get_hit(s, n->ref[0], &h->child))) return rc;
            float radians = rt_to_radians(n->f[0]);
            h->sin_t = o_sin(s->flags, radians);
            h->cos_t = o_cos(s->flags, radians);
            OAabb bb;
            if (hittable_bbox(h->child, 0.0f, 1.0f, &bb)) {
                float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
                for (int i = 0; i < 2; ++i)
                    for (int j = 0; j < 2; ++j)
                        for (int k = 0; k < 2; ++k) {
                            float fi = (float)i, fj = (float)j, fk = (float)k;
                            float x = fi * bb.mx.x + (1.0f - fi) * bb.mn.x;
                            float y = fj * bb.mx.y + (1.0f - fj) * bb.mn.y;
                            float z = fk * bb.mx.z + (1.0f - fk) * bb.mn.z;
                            float nx = h->cos_t * x + h->sin_t * z;
                            float nz = -h->sin_t * x + h->cos_t * z;
                            float tester[3] = {nx, y, nz};
                            for (int c = 0; c < 2; ++c) {
                                mn[c] = rs_min(mn[c], tester[c]);
                                mx[c] = rs_max(mx[c], tester[c]);
                            }
                        }
                h->has_rbox = 1;
                h->rbox = aabb(v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2]));
            }
            break;
        }
        case RT_OBJ_CONSTANT_MEDIUM: { /* hittable.rs:150-174 */
            if ((rc = get_hit(s, n->ref[0], &h->child))) return rc;
            const OTex* t;
            if ((rc = get_tex(s, n->ref[1], &t))) return rc;
            h->phase.kind = RT_MAT_ISOTROPIC;
            h->phase.tex = t;
            h->neg_inv_density = -1.0f / n->f[0];
            break;
        }
        default:
            return fail(RT_ERR_INVALID, "node %d: unknown kind", idx);
    }
    *out = h;
    return 0;
}

static int scene_build(OScene* s, const rt_scene_desc* d, uint32_t flags) {
    memset(s, 0, sizeof *s);
    s->d = d;
    s->flags = flags;
    if (!d || !d->nodes || d->num_nodes == 0) return fail(RT_ERR_INVALID, "empty scene");
    s->built = (void**)calloc(d->num_nodes, sizeof(void*));
    if (!s->built) return fail(RT_ERR_OOM, "oom");
    if (d->world < 0 || (uint32_t)d->world >= d->num_nodes || d->nodes[d->world].kind != RT_OBJ_LIST)
        return fail(RT_ERR_INVALID, "world must be a LIST node");
    return get_hit(s, d->world, &s->world);
}

/* ------------------------------------------------------------------------- */
/* Hittable::hit                                                              */
/* ------------------------------------------------------------------------- */
static int hittable_hit(const OHit* h, const ORay* r, float tmin, float tmax, OCtx* c, ORec* rec);

/* src/geometry/sphere.rs:49-103 — quadratic in f64 */
static int sphere_hit(const OHit* h, const ORay* r, float tmin, float tmax, OCtx* c, ORec* rec) {
    c->cnt->sphere_tests++;
    double dx = r->d.x, dy = r->d.y, dz = r->d.z;
    double ox = r->o.x, oy = r->o.y, oz = r->o.z;
    double cx = h->f[0], cy = h->f[1], cz = h->f[2];
    double radius = h->f[3];
    double ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    double a = (dx * dx + dy * dy) + dz * dz;
    double half_b = (ocx * dx + ocy * dy) + ocz * dz;
    double cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - radius * radius;
    double disc = half_b * half_b - a * cc;
    if (signbit(disc)) return 0;
    double sq = sqrt(disc);
    double root = (-half_b - sq) / a;
    if (root < (double)tmin || (double)tmax < root) {
        root = (-half_b + sq) / a;
        if (root < (double)tmin || (double)tmax < root) return 0;
    }
    float t = (float)root;
    V3 p = ray_at(r, t);
    V3 n = vdivs(vsub(p, v3(h->f[0], h->f[1], h->f[2])), h->f[3]);
    float u, v;
    sphere_uv(c->flags, n, &u, &v);
    rec_new(rec, r, n, t, u, v, h->mat);
    return 1;
}

/* src/geometry/moving_sphere.rs:54-84 — f32 */
static int msphere_hit(const OHit* h, const ORay* r, float tmin, float tmax, OCtx* c, ORec* rec) {
    c->cnt->msphere_tests++;
    float radius = h->f[8];
    V3 oc = vsub(r->o, msphere_center(h, r->time));
    float a = vdot(r->d, r->d);
    float half_b = vdot(oc, r->d);
    float cc = vdot(oc, oc) - radius * radius;
    float disc = half_b * half_b - a * cc;
    if (signbit(disc)) return 0;
    float sq = __builtin_sqrtf(disc);
    float root = (-half_b - sq) / a;
    if (root < tmin || tmax < root) {
        root = (-half_b + sq) / a;
        if (root < tmin || tmax < root) return 0;
    }
    V3 p = ray_at(r, root);
    V3 n = vdivs(vsub(p, msphere_center(h, r->time)), radius);
    float u, v;
    sphere_uv(c->flags, n, &u, &v);
    rec_new(rec, r, n, root, u, v, h->mat);
    return 1;
}

/* src/geometry/rectangle.rs:36-65, 98-127, 160-189 */
static int rect_hit(const OHit* h, const ORay* r, float tmin, float tmax, OCtx* c, ORec* rec) {
    c->cnt->rect_tests++;
    float x0 = h->f[0], x1 = h->f[1], y0 = h->f[2], y1 = h->f[3], k = h->f[4];
    float t, x, y;
    V3 n;
    if (h->kind == RT_OBJ_XY_RECT) {
        t = (k - r->o.z) / r->d.z;
        if (t < tmin || t > tmax) return 0;
        x = r->o.x + t * r->d.x;
        y = r->o.y + t * r->d.y;
        n = v3(0.0f, 0.0f, 1.0f);
    } else if (h->kind == RT_OBJ_XZ_RECT) {
        t = (k - r->o.y) / r->d.y;
        if (t < tmin || t > tmax) return 0;
        x = r->o.x + t * r->d.x;
        y = r->o.z + t * r->d.z;
        n = v3(0.0f, 1.0f, 0.0f);
    } else {
        t = (k - r->o.x) / r->d.x;
        if (t < tmin || t > tmax) return 0;
        x = r->o.y + t * r->d.y;
        y = r->o.z + t * r->d.z;
        n = v3(1.0f, 0.0f, 0.0f);
    }
    if (x < x0 || x > x1 || y < y0 || y > y1) return 0;
    float u = (x - x0) / (x1 - x0);
    float v = (y - y0) / (y1 - y0);
    rec_new(rec, r, n, t, u, v, h->mat);
    return 1;
}

/* src/geometry/triangle.rs:32-92 (Moller-Trumbore) */
static int tri_hit(const OHit* h, const ORay* r, float tmin, float tmax, OCtx* c, ORec* rec) {
    c->cnt->tri_tests++;
    const float eps = 0.0000001f;
    V3 v0 = v3(h->f[0], h->f[1], h->f[2]);
    V3 v1 = v3(h->f[3], h->f[4], h->f[5]);
    V3 v2 = v3(h->f[6], h->f[7], h->f[8]);
    V3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
    V3 hh = vcross(r->d, e2);
    float a = vdot(e1, hh);
    if (a > -eps && a < eps) return 0;
    float f = 1.0f / a;
    V3 s = vsub(r->o, v0);
    float u = f * vdot(s, hh);
    if (u < 0.0f || u > 1.0f) return 0;
    V3 q = vcross(s, e1);
    float v = f * vdot(r->d, q);
    if (v < 0.0f || u + v > 1.0f) return 0;
    float t = f * vdot(e2, q);
    if (t < tmin || t > tmax) return 0;
    if (!(t > eps)) return 0;
    V3 n = vnorm(vcross(e1, e2));
    rec_new(rec, r, n, t, 0.0f, 0.0f, h->mat);
    return 1;
}

/* src/hittable.rs:100-118 (later objects win ties: `t > t_max` rejects) */
static int list_hit(const OHit* const* items, int n, const ORay* r, float tmin, float tmax, OCtx* c,
                    ORec* rec) {
    float closest = tmax;
    int any = 0;
    ORec tmp;
    for (int i = 0; i < n; ++i) {
        if (hittable_hit(items[i], r, tmin, closest, c, &tmp)) {
            closest = tmp.t;
            *rec = tmp;
            any = 1;
        }
    }
    return any;
}

/* src/bvh.rs:363-417, the exact (no predictor) branch of Bvh::hit (:212-217) */
static int bvh_node_hit(const OBvh* b, int idx, const ORay* r, float tmin, float tmax, OCtx* c,
                        ORec* rec) {
    const OBvhNode* nd = &b->nodes[idx];
    c->cnt->node_visits++;
    if (!aabb_hit(&nd->box, r, tmin, tmax)) return 0;
    ORec lrec, rrec;
    int hl = nd->left.is_index ? bvh_node_hit(b, nd->left.idx, r, tmin, tmax, c, &lrec)
                               : hittable_hit(nd->left.obj, r, tmin, tmax, c, &lrec);
    float t_max_for_right = hl ? lrec.t : tmax;
    /* quirk kept: an Index right child is searched with t_max, a leaf with t_max_for_right */
    int hr = nd->right.is_index ? bvh_node_hit(b, nd->right.idx, r, tmin, tmax, c, &rrec)
                                : hittable_hit(nd->right.obj, r, tmin, t_max_for_right, c, &rrec);
    if (!hl && !hr) return 0;
    if (hl && !hr) *rec = lrec;
    else if (!hl && hr) *rec = rrec;
    else *rec = (lrec.t < rrec.t) ? lrec : rrec;
    return 1;
}

/* src/hittable.rs:176-233 */
static int medium_hit(const OHit* h, const ORay* r, float tmin, float tmax, OCtx* c, ORec* rec) {
    c->cnt->medium_tests++;
    ORec h1, h2;
    if (!hittable_hit(h->child, r, -INFINITY, INFINITY, c, &h1)) return 0;
    if (!hittable_hit(h->child, r, h1.t + 0.0001f, INFINITY, c, &h2)) return 0;
    if (h1.t < tmin) h1.t = tmin;
    if (h2.t > tmax) h2.t = tmax;
    if (h1.t >= h2.t) return 0;
    if (h1.t < 0.0f) h1.t = 0.0f;
    float ray_length = vlen(r->d);
    float distance_inside = (h2.t - h1.t) * ray_length;
    float hit_distance = h->neg_inv_density * o_ln(c->flags, rng_std01(&c->rng));
    if (hit_distance > distance_inside) return 0;
    float t = h1.t + hit_distance / ray_length;
    rec->t = t;
    rec->p = ray_at(r, t);
    rec->n = v3(1.0f, 0.0f, 0.0f);
    rec->u = 0.0f;
    rec->v = 0.0f;
    rec->front = 1;
    rec->mat = &h->phase;
    return 1;
}

static int hittable_hit(const OHit* h, const ORay* r, float tmin, float tmax, OCtx* c, ORec* rec) {
    switch (h->kind) {
        case RT_OBJ_SPHERE: return sphere_hit(h, r, tmin, tmax, c, rec);
        case RT_OBJ_MOVING_SPHERE: return msphere_hit(h, r, tmin, tmax, c, rec);
        case RT_OBJ_XY_RECT:
        case RT_OBJ_XZ_RECT:
        case RT_OBJ_YZ_RECT: return rect_hit(h, r, tmin, tmax, c, rec);
        case RT_OBJ_TRI: return tri_hit(h, r, tmin, tmax, c, rec);
        case RT_OBJ_CUBE: /* cube.rs:84-93 */
        case RT_OBJ_LIST: return list_hit(h->items, h->nitems, r, tmin, tmax, c, rec);
        case RT_OBJ_BVH:
        case RT_OBJ_BVH_TREE: return bvh_node_hit(&h->bvh, h->bvh.root, r, tmin, tmax, c, rec);
        case RT_OBJ_TRANSLATE: { /* instance.rs:32-43 */
            ORay off = {vsub(r->o, h->disp), r->d, r->time};
            if (!hittable_hit(h->child, &off, tmin, tmax, c, rec)) return 0;
            rec->p = vadd(rec->p, h->disp);
            return 1;
        }
        case RT_OBJ_ROTATE_Y: { /* instance.rs:114-143 */
            float cs = h->cos_t, sn = h->sin_t;
            V3 o = v3(cs * r->o.x - sn * r->o.z, r->o.y, sn * r->o.x + cs * r->o.z);
            V3 d = v3(cs * r->d.x - sn * r->d.z, r->d.y, sn * r->d.x + cs * r->d.z);
            ORay rot = {o, d, r->time};
            if (!hittable_hit(h->child, &rot, tmin, tmax, c, rec)) return 0;
            V3 p = v3(cs * rec->p.x + sn * rec->p.z, rec->p.y, -sn * rec->p.x + cs * rec->p.z);
            V3 n = v3(cs * rec->n.x + sn * rec->n.z, rec->n.y, -sn * rec->n.x + cs * rec->n.z);
            rec->p = p;
            /* set_face_normal(&ray_rotated, normal) — object-space ray, world normal */
            int front = vdot(rot.d, n) < 0.0f;
            rec->n = front ? n : vneg(n);
            return 1;
        }
        case RT_OBJ_CONSTANT_MEDIUM: return medium_hit(h, r, tmin, tmax, c, rec);
        default: return 0;
    }
}

/* ------------------------------------------------------------------------- */
/* Texture::value / Material::scatter / emit                                  */
/* ------------------------------------------------------------------------- */
static V3 tex_value(const OTex* t, float u, float v, V3 p, OCtx* c) {
    for (;;) {
        switch (t->kind) {
            case RT_TEX_SOLID: /* solid_color.rs:21-25 */
                return t->color;
            case RT_TEX_CHECKER: { /* checker.rs:27-37 */
                float sines = o_sin(c->flags, t->scale * p.x) * o_sin(c->flags, t->scale * p.y) *
                              o_sin(c->flags, t->scale * p.z);
                t = signbit(sines) ? t->odd : t->even;
                continue;
            }
            case RT_TEX_MARBLE: { /* marble.rs:23-29 */
                double nz = turb_get(t->turb, (double)p.x, (double)p.y, (double)p.z);
                float s = 0.5f * (1.0f + o_sin(c->flags, t->scale * p.z + 10.0f * (float)nz));
                return v3(s, s, s);
            }
            case RT_TEX_IMAGE: { /* image_texture.rs:21-52 */
                c->cnt->texel_fetches++;
                float uu = rs_clamp(u, 0.0f, 1.0f);
                float vv = rs_clamp(v, 0.0f, 1.0f);
                vv = 1.0f - vv;
                uint32_t i = rt_f32_to_u32_sat(uu * (float)t->w);
                uint32_t j = rt_f32_to_u32_sat(vv * (float)t->h);
                if (i >= t->w) i = t->w - 1;
                if (j >= t->h) j = t->h - 1;
                const uint8_t* px = t->img + ((size_t)j * t->w + i) * 3u;
                const float cs = 1.0f / 255.0f;
                return v3((float)px[0] * cs, (float)px[1] * cs, (float)px[2] * cs);
            }
            default:
                return v3(0.0f, 0.0f, 0.0f);
        }
    }
}

/* material.rs:20-22 default emit = 0; diffuse_light.rs:34-36 */
static V3 mat_emit(const OMat* m, float u, float v, V3 p, OCtx* c) {
    if (m->kind == RT_MAT_DIFFUSE_LIGHT) return tex_value(m->tex, u, v, p, c);
    return v3(0.0f, 0.0f, 0.0f);
}

/* dialectric.rs:26-29 (powi(5) = x * ((x*x)*(x*x)), LLVM's expansion) */
static inline float reflectance(float cosv, float ref_idx) {
    float q = (1.0f - ref_idx) / (1.0f + ref_idx);
    float r0 = q * q;
    float x = 1.0f - cosv;
    float x2 = x * x;
    return r0 + (1.0f - r0) * (x * (x2 * x2));
}

static int mat_scatter(const OMat* m, const ORay* r, const ORec* rec, OCtx* c, V3* att, ORay* sc) {
    switch (m->kind) {
        case RT_MAT_LAMBERTIAN: { /* lambertian.rs:34-53 */
            V3 dir = vadd(rec->n, vnorm(random_in_unit_sphere(c)));
            if (near_zero(dir)) dir = rec->n;
            sc->o = rec->p; sc->d = dir; sc->time = r->time;
            *att = tex_value(m->tex, rec->u, rec->v, rec->p, c);
            return 1;
        }
        case RT_MAT_METAL: { /* metal.rs:25-43 */
            V3 reflected = reflect(vnorm(r->d), rec->n);
            V3 dir = vadd(reflected, vscale(m->fuzz, random_in_unit_sphere(c)));
            sc->o = rec->p; sc->d = dir; sc->time = r->time;
            *att = m->albedo;
            return vdot(dir, rec->n) > 0.0f;
        }
        case RT_MAT_DIELECTRIC: { /* dialectric.rs:32-61 */
            *att = v3(1.0f, 1.0f, 1.0f);
            float ratio = rec->front ? 1.0f / m->ior : m->ior;
            V3 ud = vnorm(r->d);
            float cos_t = rs_min(vdot(vneg(ud), rec->n), 1.0f);
            float sin_t = __builtin_sqrtf(1.0f - cos_t * cos_t);
            int cannot = ratio * sin_t > 1.0f;
            V3 dir;
            if (cannot || reflectance(cos_t, ratio) > rng_std01(&c->rng)) dir = reflect(ud, rec->n);
            else dir = refract(ud, rec->n, ratio);
            sc->o = rec->p; sc->d = dir; sc->time = r->time;
            return 1;
        }
        case RT_MAT_ISOTROPIC: { /* isotropic.rs:31-43 */
            V3 dir = random_in_unit_sphere(c);
            sc->o = rec->p; sc->d = dir; sc->time = r->time;
            *att = tex_value(m->tex, rec->u, rec->v, rec->p, c);
            return 1;
        }
        default: /* DiffuseLight: diffuse_light.rs:26-32 */
            return 0;
    }
}

/* ------------------------------------------------------------------------- */
/* Ray::ray_color (src/ray.rs:32-62)                                          */
/* ------------------------------------------------------------------------- */
static V3 ray_color_rec(const OScene* s, const ORay* ray, uint32_t depth, V3 bg, OCtx* c) {
    if (depth == 0) return v3(0.0f, 0.0f, 0.0f);
    c->cnt->segments++;
    ORec rec;
    if (!hittable_hit(s->world, ray, 0.001f, INFINITY, c, &rec)) return bg;
    c->cnt->hits++;
    V3 e = mat_emit(rec.mat, rec.u, rec.v, rec.p, c);
    V3 att;
    ORay sc;
    if (mat_scatter(rec.mat, ray, &rec, c, &att, &sc))
        return vadd(e, vmul(att, ray_color_rec(s, &sc, depth - 1, bg, c)));
    return e;
}
/* The device's order: L += T*e at each vertex, T *= attenuation (forward
 * product). Same random draws and branches as the recursion; radiance differs
 * from it only by float reassociation (checked <= 1e-5 in tests). */
#ifdef ORACLE_TRACE
static __thread int g_trace; /* diagnostic build only: get_color sets it for one (pixel, sample) */
static uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
#endif
static V3 ray_color_fwd(const OScene* s, ORay ray, uint32_t depth, V3 bg, OCtx* c) {
    V3 L = v3(0.0f, 0.0f, 0.0f), T = v3(1.0f, 1.0f, 1.0f);
    while (depth > 0) {
        c->cnt->segments++;
        ORec rec;
        int hit = hittable_hit(s->world, &ray, 0.001f, INFINITY, c, &rec);
#ifdef ORACLE_TRACE
        if (g_trace)
            fprintf(stderr, "TRACE depth %u o %08x %08x %08x d %08x %08x %08x any %d t %08x\n", depth, fbits(ray.o.x),
                   fbits(ray.o.y), fbits(ray.o.z), fbits(ray.d.x), fbits(ray.d.y), fbits(ray.d.z), hit,
                   hit ? fbits(rec.t) : 0x7f800000u);
#endif
        if (!hit) {
            L = vadd(L, vmul(T, bg));
            break;
        }
        c->cnt->hits++;
        V3 e = mat_emit(rec.mat, rec.u, rec.v, rec.p, c);
        L = vadd(L, vmul(T, e));
        V3 att;
        ORay sc;
        if (!mat_scatter(rec.mat, &ray, &rec, c, &att, &sc)) break;
        T = vmul(T, att);
        ray = sc;
        depth--;
    }
    return L;
}

/* ------------------------------------------------------------------------- */
/* Camera (src/camera.rs:44-106)                                              */
/* ------------------------------------------------------------------------- */
typedef struct {
    V3 origin, horizontal, vertical, llc, u, v;
    float lens_radius, time_low, time_scale;
} OCam;
static int camera_new(const rt_camera_desc* d, uint32_t flags, OCam* cam) {
    V3 lf = v3(d->look_from[0], d->look_from[1], d->look_from[2]);
    V3 la = v3(d->look_at[0], d->look_at[1], d->look_at[2]);
    V3 vup = v3(d->view_up[0], d->view_up[1], d->view_up[2]);
    float theta = rt_to_radians(d->vfov_deg);
    float h = o_tan(flags, theta / 2.0f);
    float vh = 2.0f * h;
    float vw = d->aspect_ratio * vh;
    V3 w = vnorm(vsub(lf, la));
    V3 u = vnorm(vcross(vup, w));
    V3 v = vcross(w, u);
    cam->origin = lf;
    cam->horizontal = vscale(d->focus_dist * vw, u);
    cam->vertical = vscale(d->focus_dist * vh, v);
    cam->llc = vsub(vsub(vsub(lf, vdivs(cam->horizontal, 2.0f)), vdivs(cam->vertical, 2.0f)),
                    vscale(d->focus_dist, w));
    cam->u = u;
    cam->v = v;
    cam->lens_radius = d->aperture / 2.0f;
    cam->time_low = d->time0;
    if (!uniform_inclusive(d->time0, d->time1, &cam->time_scale))
        return fail(RT_ERR_INVALID, "Uniform::new_inclusive called with `low > high`");
    return 0;
}
/* A constructed Camera (src/camera.rs:6-27) as Renderer::render receives it. */
static int camera_from_fields(const rt_camera* k, OCam* cam) {
    cam->origin = v3(k->origin[0], k->origin[1], k->origin[2]);
    cam->horizontal = v3(k->horizontal[0], k->horizontal[1], k->horizontal[2]);
    cam->vertical = v3(k->vertical[0], k->vertical[1], k->vertical[2]);
    cam->llc = v3(k->lower_left_corner[0], k->lower_left_corner[1], k->lower_left_corner[2]);
    cam->u = v3(k->u[0], k->u[1], k->u[2]);
    cam->v = v3(k->v[0], k->v[1], k->v[2]);
    cam->lens_radius = k->lens_radius;
    cam->time_low = k->time_start;
    if (!uniform_inclusive(k->time_start, k->time_end, &cam->time_scale))
        return fail(RT_ERR_INVALID, "Uniform::new_inclusive called with `low > high`");
    return 0;
}
void oracle_camera_basis(const rt_camera_desc* d, float out[21]) {
    OCam c;
    memset(&c, 0, sizeof c);
    camera_new(d, 0, &c);
    V3 vs[6] = {c.origin, c.horizontal, c.vertical, c.llc, c.u, c.v};
    for (int i = 0; i < 6; ++i) {
        out[3 * i] = vs[i].x;
        out[3 * i + 1] = vs[i].y;
        out[3 * i + 2] = vs[i].z;
    }
    out[18] = c.lens_radius;
    out[19] = c.time_low;
    out[20] = c.time_scale;
}
static ORay camera_get_ray(const OCam* cam, float s, float t, OCtx* c) {
    V3 rd = vscale(cam->lens_radius, random_in_unit_disk(c));
    V3 offset = vadd(vscale(rd.x, cam->u), vscale(rd.y, cam->v));
    ORay r;
    r.o = vadd(cam->origin, offset);
    r.d = vsub(vsub(vadd(vadd(cam->llc, vscale(s, cam->horizontal)), vscale(t, cam->vertical)), cam->origin),
               offset);
    float v01 = f32_from_1_2(rng_u32(&c->rng)) - 1.0f; /* UniformFloat::sample */
    r.time = v01 * cam->time_scale + cam->time_low;
    return r;
}

/* ------------------------------------------------------------------------- */
/* Renderer (src/renderer.rs)                                                 */
/* ------------------------------------------------------------------------- */
/* Tile::tile, renderer.rs:242-296 */
uint32_t oracle_tile(uint32_t w, uint32_t h, uint32_t tw, uint32_t th, rt_tile* out, uint32_t cap) {
    if (tw == 0 || th == 0) return 0;
    uint32_t nh = w / tw, rh = w % tw, nv = h / th, rv = h % th, n = 0;
#define PUSH(W_, H_, X_, Y_)                                   \
    do {                                                       \
        if (n < cap) {                                         \
            out[n].width = (W_); out[n].height = (H_);         \
            out[n].x_start = (X_); out[n].y_start = (Y_);      \
        }                                                      \
        n++;                                                   \
    } while (0)
    for (uint32_t ty = 0; ty < nv; ++ty) {
        for (uint32_t tx = 0; tx < nh; ++tx) PUSH(tw, th, tx * tw, ty * th);
        if (rh > 0) PUSH(rh, th, nh * tw, ty * th);
    }
    if (rv > 0)
        for (uint32_t tx = 0; tx < nh; ++tx) PUSH(tw, rv, tx * tw, nv * th);
    if (rh > 0 && rv > 0) PUSH(rh, rv, nh * tw, nv * th);
#undef PUSH
    return n;
}

typedef struct {
    const OScene* scene;
    const OCam* cam;
    const rt_render_params* p;
    const rt_tile* tiles;
    uint32_t ntiles;
    uint32_t next; /* atomic */
    float* out;
    uint32_t flags;
    pthread_mutex_t mu;
    oracle_counters total;
} OJob;

static inline int in_shard(const rt_render_params* p, uint32_t x, uint32_t y) {
    if (p->shard_count <= 1) return 1;
    uint32_t nbx = (p->width + 7) / 8;
    uint32_t b = (y / 8) * nbx + (x / 8);
    return b % p->shard_count == p->shard_index;
}

/* Renderer::get_color, renderer.rs:129-149 */
static V3 get_color(const OJob* j, uint32_t x, uint32_t y, OCtx* c) {
    const rt_render_params* p = j->p;
    V3 acc = v3(0.0f, 0.0f, 0.0f);
    V3 bg = v3(p->background[0], p->background[1], p->background[2]);
    uint32_t pixel = y * p->width + x;
    for (uint32_t s = 0; s < p->samples_per_pixel; ++s) {
        rng_init(&c->rng, p->seed, pixel, p->sample_base + s);
#ifdef ORACLE_TRACE
        g_trace = pixel == ORACLE_TRACE_PIXEL && p->sample_base + s == ORACLE_TRACE_SAMPLE;
#endif
        c->cnt->samples++;
        float u = ((float)x + rng_std01(&c->rng)) / (float)(p->width - 1);
        float v = ((float)y + rng_std01(&c->rng)) / (float)(p->height - 1);
        ORay ray = camera_get_ray(j->cam, u, v, c);
        V3 L = (j->flags & ORACLE_FLAG_RECURSIVE) ? ray_color_rec(j->scene, &ray, p->max_depth, bg, c)
                                                  : ray_color_fwd(j->scene, ray, p->max_depth, bg, c);
        acc = vadd(acc, L);
    }
    return vdivs(acc, (float)p->samples_per_pixel);
}

static void* worker(void* arg) {
    OJob* j = (OJob*)arg;
    oracle_counters cnt;
    memset(&cnt, 0, sizeof cnt);
    OCtx c;
    c.cnt = &cnt;
    c.flags = j->flags;
    for (;;) {
        uint32_t t = __atomic_fetch_add(&j->next, 1u, __ATOMIC_RELAXED);
        if (t >= j->ntiles) break;
        const rt_tile* tl = &j->tiles[t];
        for (uint32_t yy = 0; yy < tl->height; ++yy)
            for (uint32_t xx = 0; xx < tl->width; ++xx) {
                uint32_t x = tl->x_start + xx, y = tl->y_start + yy;
                if (!in_shard(j->p, x, y)) continue;
                V3 col = get_color(j, x, y, &c);
                float* o = j->out + ((size_t)y * j->p->width + x) * 3u;
                o[0] = col.x; o[1] = col.y; o[2] = col.z;
            }
    }
    pthread_mutex_lock(&j->mu);
    uint64_t* dst = &j->total.samples;
    const uint64_t* src = &cnt.samples;
    for (int i = 0; i < 10; ++i) dst[i] += src[i];
    pthread_mutex_unlock(&j->mu);
    return NULL;
}

static int check_params(const rt_render_params* p) {
    if (!p) return fail(RT_ERR_INVALID, "params is NULL");
    if (p->width == 0 || p->height == 0) return fail(RT_ERR_INVALID, "empty image");
    if (p->samples_per_pixel == 0) return fail(RT_ERR_INVALID, "samples_per_pixel must be > 0");
    if (p->tile_width == 0 || p->tile_height == 0) return fail(RT_ERR_INVALID, "tile size must be >= 1");
    if (p->shard_count > 1 && p->shard_index >= p->shard_count) return fail(RT_ERR_INVALID, "shard_index >= shard_count");
    return 0;
}

static int render_with(const rt_scene_desc* scene, const rt_camera_desc* camera, const rt_camera* fields,
                       const rt_render_params* p, const oracle_options* opt, float* out, oracle_counters* counters) {
    int rc = check_params(p);
    if (rc) return rc;
    if ((!camera && !fields) || !out) return fail(RT_ERR_INVALID, "camera/out is NULL");
    uint32_t flags = opt ? opt->flags : 0u;
    OScene s;
    if ((rc = scene_build(&s, scene, flags))) {
        scene_free(&s);
        return rc;
    }
    OCam cam;
    if ((rc = camera ? camera_new(camera, flags, &cam) : camera_from_fields(fields, &cam))) {
        scene_free(&s);
        return rc;
    }
    uint32_t ntiles = oracle_tile(p->width, p->height, p->tile_width, p->tile_height, NULL, 0);
    rt_tile* tiles = (rt_tile*)malloc(sizeof(rt_tile) * (size_t)ntiles);
    if (!tiles) {
        scene_free(&s);
        return fail(RT_ERR_OOM, "oom");
    }
    oracle_tile(p->width, p->height, p->tile_width, p->tile_height, tiles, ntiles);
    OJob j;
    memset(&j, 0, sizeof j);
    j.scene = &s;
    j.cam = &cam;
    j.p = p;
    j.tiles = tiles;
    j.ntiles = ntiles;
    j.out = out;
    j.flags = flags;
    pthread_mutex_init(&j.mu, NULL);
    long ncpu = sysconf(_SC_NPROCESSORS_ONLN);
    uint32_t nt = (opt && opt->num_threads) ? opt->num_threads : (uint32_t)(ncpu > 0 ? ncpu : 1);
    if (nt > ntiles) nt = ntiles;
    if (nt < 1) nt = 1;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nt);
    uint32_t started = 0;
    for (uint32_t i = 1; th && i < nt; ++i)
        if (pthread_create(&th[i], NULL, worker, &j) == 0) started++;
        else break;
    worker(&j);
    for (uint32_t i = 1; i <= started; ++i) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    free(tiles);
    pthread_mutex_destroy(&j.mu);
    scene_free(&s);
    if (counters) {
        *counters = j.total;
        counters->seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        counters->threads = started + 1;
    }
    return 0;
}

int oracle_render(const rt_scene_desc* scene, const rt_camera_desc* camera, const rt_render_params* p,
                  const oracle_options* opt, float* out, oracle_counters* counters) {
    return render_with(scene, camera, NULL, p, opt, out, counters);
}

int oracle_render_camera(const rt_scene_desc* scene, const rt_camera* camera, const rt_render_params* p,
                         const oracle_options* opt, float* out, oracle_counters* counters) {
    if (!camera) return fail(RT_ERR_INVALID, "camera is NULL");
    return render_with(scene, NULL, camera, p, opt, out, counters);
}

int oracle_sample(const rt_scene_desc* scene, const rt_camera_desc* camera, const rt_render_params* p,
                  uint32_t flags, uint32_t x, uint32_t y, uint32_t sample, float rgb[3]) {
    int rc = check_params(p);
    if (rc) return rc;
    OScene s;
    if ((rc = scene_build(&s, scene, flags))) {
        scene_free(&s);
        return rc;
    }
    OCam cam;
    if ((rc = camera_new(camera, flags, &cam))) {
        scene_free(&s);
        return rc;
    }
    oracle_counters cnt;
    memset(&cnt, 0, sizeof cnt);
    OCtx c;
    c.cnt = &cnt;
    c.flags = flags;
    rng_init(&c.rng, p->seed, y * p->width + x, p->sample_base + sample);
    float u = ((float)x + rng_std01(&c.rng)) / (float)(p->width - 1);
    float v = ((float)y + rng_std01(&c.rng)) / (float)(p->height - 1);
    ORay ray = camera_get_ray(&cam, u, v, &c);
    V3 bg = v3(p->background[0], p->background[1], p->background[2]);
    V3 L = (flags & ORACLE_FLAG_RECURSIVE) ? ray_color_rec(&s, &ray, p->max_depth, bg, &c)
                                           : ray_color_fwd(&s, ray, p->max_depth, bg, &c);
    rgb[0] = L.x; rgb[1] = L.y; rgb[2] = L.z;
    scene_free(&s);
    return 0;
}

/* Host evaluation of the numeric spec / IEEE primitives, for the device
 * bit-exactness checks (ops as rt_device_numeric_eval). */
void oracle_numeric_eval(int op, const double* a, const double* b, double* out, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) {
        double x = a[i], y = b ? b[i] : 0.0, r = 0.0;
        switch (op) {
            case 0: r = sqrt(x); break;
            case 1: r = (double)__builtin_sqrtf((float)x); break;
            case 2: r = (double)((float)x / (float)y); break;
            case 3: r = (double)rt_sinf((float)x); break;
            case 4: r = (double)rt_acosf((float)x); break;
            case 5: r = (double)rt_atan2f((float)x, (float)y); break;
            case 6: r = (double)rt_logf((float)x); break;
            case 7: r = x / y; break;
            case 8: r = (double)rt_cosf((float)x); break;
            case 9: r = (double)rt_tanf((float)x); break;
            default: r = 0.0; break;
        }
        out[i] = r;
    }
}
