/*
 * prebuilt_tree.c — the drop-in boundary exercised from C (not ctypes).
 *
 * The reference's Renderer::render (src/renderer.rs:42-52) receives a built
 * `Camera` (its nine fields, src/camera.rs:6-27) and a world whose Bvh objects
 * are already built node arrays (src/bvh.rs:38-43, BvhNode :228-235). This
 * program hands the library exactly that: RT_OBJ_BVH_TREE nodes whose trees it
 * builds itself with a different algorithm than Bvh::new (longest-axis centroid
 * median, so the shapes and DFS-rank ties are the caller's, not the library's),
 * and an explicit rt_camera. It renders through rt_render_camera and requires the
 * image and the segment count to equal the CPU oracle's (oracle_render_camera,
 * fed the same descriptor) bit for bit. It also checks that rt_render with the
 * Camera::new arguments equals rt_render_camera with rt_camera_new's fields.
 *
 * Test infrastructure: built by tests/capi/Makefile, run by
 * tests/test_capi_c.py (-m gpu). Exit status 0 = pass.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rt.h"
#include "../../oracle/oracle.h"

#define MAX_NODES 4096
#define MAX_BVH 4096

static rt_node nodes[MAX_NODES];
static int nn = 0;
static int32_t items[MAX_NODES];
static int ni = 0;
static rt_bvh_node bvh[MAX_BVH];
static int nb = 0;

static uint64_t lcg = 0x9e3779b97f4a7c15ull;
static float frand(void) { /* [0, 1) */
    lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
    return (float)(lcg >> 40) / 16777216.0f;
}

static int add(uint32_t kind, const float* f, int nf, int r0, int r1, int r2, uint64_t seed) {
    rt_node* n = &nodes[nn];
    memset(n, 0, sizeof *n);
    n->kind = kind;
    n->ref[0] = r0;
    n->ref[1] = r1;
    n->ref[2] = r2;
    for (int i = 0; i < nf; ++i) n->f[i] = f[i];
    n->seed = seed;
    return nn++;
}
static int solid(float r, float g, float b) { float f[3] = {r, g, b}; return add(RT_TEX_SOLID, f, 3, -1, -1, -1, 0); }
static int lambertian(int tex) { return add(RT_MAT_LAMBERTIAN, NULL, 0, tex, -1, -1, 0); }
static int metal(float r, float g, float b, float fuzz) { float f[4] = {r, g, b, fuzz}; return add(RT_MAT_METAL, f, 4, -1, -1, -1, 0); }
static int dielectric(float ior) { return add(RT_MAT_DIELECTRIC, &ior, 1, -1, -1, -1, 0); }
static int sphere(float x, float y, float z, float r, int m) { float f[4] = {x, y, z, r}; return add(RT_OBJ_SPHERE, f, 4, m, -1, -1, 0); }
static int cube(float x0, float y0, float z0, float x1, float y1, float z1, int m) {
    float f[6] = {x0, y0, z0, x1, y1, z1};
    return add(RT_OBJ_CUBE, f, 6, m, -1, -1, 0);
}
static int tri(const float* p, int m) { return add(RT_OBJ_TRI, p, 9, m, -1, -1, 0); }
static int list(const int* objs, int n) {
    int first = ni;
    for (int i = 0; i < n; ++i) items[ni++] = objs[i];
    return add(RT_OBJ_LIST, NULL, 0, first, n, -1, 0);
}

/* Hittable::bounding_box(0, 1) of a primitive, in f32 exactly like the reference
 * (sphere.rs:105-109, cube.rs:95-97, triangle.rs:94-107 with f32::EPSILON). */
static void prim_box(int idx, float mn[3], float mx[3]) {
    const rt_node* n = &nodes[idx];
    const float* f = n->f;
    if (n->kind == RT_OBJ_SPHERE) {
        for (int k = 0; k < 3; ++k) { mn[k] = f[k] - f[3]; mx[k] = f[k] + f[3]; }
    } else if (n->kind == RT_OBJ_CUBE) {
        for (int k = 0; k < 3; ++k) { mn[k] = f[k]; mx[k] = f[3 + k]; }
    } else { /* RT_OBJ_TRI */
        const float eps = 1.1920929e-07f;
        for (int k = 0; k < 3; ++k) {
            float a = fminf(f[k], fminf(f[3 + k], f[6 + k])), b = fmaxf(f[k], fmaxf(f[3 + k], f[6 + k]));
            mn[k] = a - eps;
            mx[k] = b + eps;
        }
    }
}

typedef struct { int obj; float mn[3], mx[3], c[3]; } Item;
static int sort_axis;
static int cmp_c(const void* a, const void* b) {
    const Item* x = (const Item*)a;
    const Item* y = (const Item*)b;
    if (x->c[sort_axis] < y->c[sort_axis]) return -1;
    if (x->c[sort_axis] > y->c[sort_axis]) return 1;
    return x->obj - y->obj;
}

/* Builds a subtree over it[0..n) into bvh[first + ...] in postorder (children
 * before parents, like BvhNode::new_helper pushes them); returns the node index
 * relative to `first`. The split is the caller's own: longest centroid axis. */
static int build(Item* it, int n, int first) {
    rt_bvh_node node;
    memset(&node, 0, sizeof node);
    node.parent = -1;
    if (n <= 2) {
        node.flags = RT_BVH_LEFT_HITTABLE | RT_BVH_RIGHT_HITTABLE;
        node.left = it[0].obj;
        node.right = n == 2 ? it[1].obj : it[0].obj; /* 1-object node repeats it (bvh.rs:261-264) */
        for (int k = 0; k < 3; ++k) {
            node.bbox_min[k] = n == 2 ? fminf(it[0].mn[k], it[1].mn[k]) : it[0].mn[k];
            node.bbox_max[k] = n == 2 ? fmaxf(it[0].mx[k], it[1].mx[k]) : it[0].mx[k];
        }
    } else {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k) { lo[k] = fminf(lo[k], it[i].c[k]); hi[k] = fmaxf(hi[k], it[i].c[k]); }
        sort_axis = 0;
        for (int k = 1; k < 3; ++k)
            if (hi[k] - lo[k] > hi[sort_axis] - lo[sort_axis]) sort_axis = k;
        qsort(it, (size_t)n, sizeof(Item), cmp_c);
        int mid = n / 3 + 1; /* deliberately unbalanced */
        int l = build(it, mid, first), r = build(it + mid, n - mid, first);
        node.left = l;
        node.right = r;
        for (int k = 0; k < 3; ++k) { /* Aabb::union (aabb.rs:43-62) */
            node.bbox_min[k] = fminf(bvh[first + l].bbox_min[k], bvh[first + r].bbox_min[k]);
            node.bbox_max[k] = fmaxf(bvh[first + l].bbox_max[k], bvh[first + r].bbox_max[k]);
        }
    }
    int me = nb - first;
    bvh[nb++] = node;
    if (node.flags == 0) {
        bvh[first + node.left].parent = me;
        bvh[first + node.right].parent = me;
    }
    return me;
}

static int bvh_tree(const int* objs, int n) {
    Item* it = (Item*)malloc(sizeof(Item) * (size_t)n);
    for (int i = 0; i < n; ++i) {
        it[i].obj = objs[i];
        prim_box(objs[i], it[i].mn, it[i].mx);
        for (int k = 0; k < 3; ++k) it[i].c[k] = 0.5f * (it[i].mn[k] + it[i].mx[k]);
    }
    int first = nb;
    int root = build(it, n, first);
    free(it);
    float f[3] = {0.0f, 1.0f, 0.0f};
    return add(RT_OBJ_BVH_TREE, f, 3, first, nb - first, root, 0);
}

static int fail(const char* what) {
    fprintf(stderr, "prebuilt_tree: %s: %s\n", what, rt_last_error());
    return 1;
}

int main(void) {
    if (rt_abi_version() != RT_ABI_VERSION) return fail("ABI version");
    /* world: ground, a tree of spheres and cubes (prunable), a tree of triangles
     * (unprunable), a glass sphere with a medium inside, a light-ish metal */
    int ground = lambertian(solid(0.5f, 0.5f, 0.5f));
    int glass = dielectric(1.5f);
    int world[8], nw = 0;
    world[nw++] = sphere(0.0f, -1000.0f, 0.0f, 1000.0f, ground);
    int objs[400], no = 0;
    for (int i = 0; i < 160; ++i) {
        float x = -8.0f + 16.0f * frand(), z = -8.0f + 16.0f * frand(), r = 0.15f + 0.25f * frand();
        int m = i % 3 == 0 ? metal(frand(), frand(), frand(), 0.3f * frand())
                           : (i % 7 == 0 ? glass : lambertian(solid(frand(), frand(), frand())));
        objs[no++] = sphere(x, r, z, r, m);
    }
    for (int i = 0; i < 40; ++i) {
        float x = -8.0f + 16.0f * frand(), z = -8.0f + 16.0f * frand(), s = 0.2f + 0.4f * frand();
        objs[no++] = cube(x, 0.0f, z, x + s, 2.0f * s, z + s, lambertian(solid(frand(), frand(), frand())));
    }
    world[nw++] = bvh_tree(objs, no);
    int tris[200], nt = 0;
    int white = lambertian(solid(0.73f, 0.73f, 0.73f));
    for (int i = 0; i < 120; ++i) { /* a fan of triangles standing on the ground */
        float a = 6.2831853f * (float)i / 120.0f, b = 6.2831853f * (float)(i + 1) / 120.0f;
        float p[9] = {3.0f * cosf(a) + 1.0f, 0.01f, 3.0f * sinf(a) - 1.0f, 3.0f * cosf(b) + 1.0f, 0.01f,
                      3.0f * sinf(b) - 1.0f, 1.0f, 1.5f + 0.5f * frand(), -1.0f};
        tris[nt++] = tri(p, white);
    }
    world[nw++] = bvh_tree(tris, nt);
    int ball = sphere(0.0f, 1.0f, 0.0f, 1.0f, glass);
    world[nw++] = ball;
    {
        float f[1] = {0.7f};
        world[nw++] = add(RT_OBJ_CONSTANT_MEDIUM, f, 1, sphere(0.0f, 1.0f, 0.0f, 0.95f, glass), solid(0.2f, 0.4f, 0.9f),
                          -1, 0);
    }
    int wl = list(world, nw);

    rt_scene_desc d;
    memset(&d, 0, sizeof d);
    d.nodes = nodes;
    d.num_nodes = (uint32_t)nn;
    d.world = wl;
    d.list_items = items;
    d.num_list_items = (uint32_t)ni;
    d.bvh_nodes = bvh;
    d.num_bvh_nodes = (uint32_t)nb;

    /* An explicit Camera: the nine fields, not Camera::new's arguments (a slightly
     * sheared basis no look_from / look_at would give, and a lens). */
    rt_camera cam = {{13.0f, 2.0f, 3.0f},   {-2.6f, 0.0f, 11.4f}, {-0.31f, 6.5f, 0.15f},
                     {2.2f, -3.1f, -7.1f},  {-0.225f, 0.0f, 0.974f}, {-0.047f, 0.998f, 0.011f},
                     0.05f, 0.0f, 1.0f};

    rt_render_params p;
    memset(&p, 0, sizeof p);
    p.width = 96;
    p.height = 64;
    p.samples_per_pixel = 8;
    p.max_depth = 12;
    p.tile_width = p.tile_height = 8;
    p.seed = 7;
    p.background[0] = 0.7f;
    p.background[1] = 0.8f;
    p.background[2] = 1.0f;

    const size_t floats = (size_t)p.width * p.height * 3;
    float* got = (float*)calloc(floats, sizeof(float));
    float* want = (float*)calloc(floats, sizeof(float));
    rt_scene_handle h = NULL;
    if (rt_scene_upload(&d, 0, &h)) return fail("rt_scene_upload");
    rt_stats st;
    if (rt_render_camera(h, &cam, &p, got, &st)) return fail("rt_render_camera");
    oracle_counters oc;
    oracle_options oo = {0u, 0u};
    if (oracle_render_camera(&d, &cam, &p, &oo, want, &oc)) {
        fprintf(stderr, "oracle: %s\n", oracle_last_error());
        return 1;
    }
    size_t diff = 0;
    for (size_t i = 0; i < floats; ++i)
        if (memcmp(&got[i], &want[i], sizeof(float)) != 0) ++diff;
    printf("prebuilt trees: %d BvhNodes; camera basis render %ux%u x %u spp: %zu of %zu values differ, "
           "segments %llu (oracle %llu)\n",
           nb, p.width, p.height, p.samples_per_pixel, diff, floats, (unsigned long long)st.segments,
           (unsigned long long)oc.segments);
    int bad = diff != 0 || st.segments != oc.segments;

    /* rt_render(Camera::new args) == rt_render_camera(rt_camera_new(args)) */
    rt_camera_desc a = {{478.0f, 278.0f, -600.0f}, {278.0f, 278.0f, 0.0f}, {0.0f, 1.0f, 0.0f}, 40.0f, 1.5f, 0.1f,
                        10.0f, 0.0f, 1.0f};
    rt_camera built;
    if (rt_camera_new(&a, &built)) return fail("rt_camera_new");
    memset(got, 0, floats * sizeof(float));
    memset(want, 0, floats * sizeof(float));
    if (rt_render(h, &a, &p, got, NULL)) return fail("rt_render");
    if (rt_render_camera(h, &built, &p, want, NULL)) return fail("rt_render_camera");
    size_t diff2 = 0;
    for (size_t i = 0; i < floats; ++i)
        if (memcmp(&got[i], &want[i], sizeof(float)) != 0) ++diff2;
    printf("rt_render(Camera::new args) vs rt_render_camera(rt_camera_new): %zu values differ\n", diff2);
    bad |= diff2 != 0;

    /* a malformed tree is reported, not aborted on: a child box outside its parent's */
    rt_bvh_node saved = bvh[nb - 1];
    bvh[nb - 1].bbox_max[1] = bvh[nb - 1].bbox_min[1];
    rt_scene_handle h2 = NULL;
    int rc = rt_scene_upload(&d, 0, &h2);
    printf("shrunken root box: rt_scene_upload -> %d (%s)\n", rc, rt_last_error());
    bad |= rc != RT_ERR_UNSUPPORTED;
    bvh[nb - 1] = saved;
    rt_scene_free(h2);
    rt_scene_free(h);
    free(got);
    free(want);
    printf(bad ? "FAIL\n" : "PASS\n");
    return bad;
}
