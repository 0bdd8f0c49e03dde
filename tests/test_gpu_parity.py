"""HIP path vs the CPU oracle, through the C ABI, on a real MI355X.

Bar: BIT-EXACT (np.testing.assert_array_equal, NaNs included) — the kernel and
the oracle consume the same Philox stream and evaluate the same IEEE
operations in the same order (Parity). North-star tolerance
(L-inf < 1e-3 on clamp01) is therefore met with zero margin used; the tests
that compare differently-reassociated quantities state their tolerance inline.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
CASES = json.load(open(os.path.join(GOLDEN, "cases.json")))


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "renders.npz"))


def gpu_render(rt, scene, camera, params):
    ds = rt.DeviceScene(scene)
    try:
        img, st = ds.render(camera, params)
    finally:
        ds.close()
    return img, st


# --- numerics -----------------------------------------------------------------
def test_device_ieee_and_spec_match_host_bit_for_bit(rt, orc):
    rng = np.random.default_rng(3)
    n = 200000
    cases = {
        0: (np.concatenate([rng.uniform(0, 1e6, n), rng.uniform(0, 1e-3, n), 10.0 ** rng.uniform(-300, 300, n)]), None),
        1: (rng.uniform(0, 1e6, n).astype(np.float32).astype(np.float64), None),
        2: (rng.uniform(-1e3, 1e3, n).astype(np.float32).astype(np.float64),
            rng.uniform(-10, 10, n).astype(np.float32).astype(np.float64)),
        3: (rng.uniform(-1e4, 1e4, n).astype(np.float32).astype(np.float64), None),
        4: (rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64), None),
        5: (rng.uniform(-5, 5, n).astype(np.float32).astype(np.float64),
            rng.uniform(-5, 5, n).astype(np.float32).astype(np.float64)),
        6: (np.concatenate([rng.uniform(0, 1, n), np.arange(0, 1 << 16) * 2.0 ** -24]).astype(np.float32)
            .astype(np.float64), None),
        7: (rng.uniform(-1e3, 1e3, n), rng.uniform(-10, 10, n)),
    }
    for op, (a, b) in cases.items():
        dev = rt.numeric_eval(op, a, b)
        host = orc.numeric_eval(op, a, b)
        mism = np.flatnonzero(dev.view(np.uint64) != host.view(np.uint64))
        assert mism.size == 0, (op, mism[:5], a[mism[:5]], dev[mism[:5]], host[mism[:5]])


# --- golden fixtures ------------------------------------------------------------
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_matches_golden(name, golden, rt):
    from golden.make_golden import case_setup
    cfg, scene, params = case_setup(rt, CASES[name])
    img, st = gpu_render(rt, scene, cfg.camera(), params)
    np.testing.assert_array_equal(img, golden[name])
    assert st["samples"] == cfg.width * cfg.height * cfg.spp


@pytest.mark.parametrize("name", ["c3_showcase", "c5_cornell_smoke", "c4_bunny", "c1_random_spheres"])
def test_exact_and_pruned_bvh_agree(name, golden, rt):
    from golden.make_golden import case_setup
    c = dict(CASES[name])
    c["exact_bvh"] = not c.get("exact_bvh", False)
    cfg, scene, params = case_setup(rt, c)
    img, _ = gpu_render(rt, scene, cfg.camera(), params)
    np.testing.assert_array_equal(img, golden[name])


# --- live oracle comparisons ------------------------------------------------------
def setup(rt, cfg_name, width, spp, seed=1, scene_seed=None, **kw):
    cfg = rt.CONFIGS[cfg_name].scaled(width, spp)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed if scene_seed is None else scene_seed)
    params = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(), seed=seed, **kw)
    return cfg, scene, params


@pytest.mark.parametrize("cfg_name,width,spp,seed,scene_seed", [
    ("C1", 37, 3, 99, 5), ("C2", 29, 2, 7, 11), ("C3", 41, 3, 12345, 3), ("C4", 33, 2, 5, 20231),
    ("C5", 35, 3, 2 ** 40 + 17, 20231)])
def test_gpu_matches_oracle_other_seeds_and_ragged_sizes(cfg_name, width, spp, seed, scene_seed, rt, orc):
    cfg, scene, params = setup(rt, cfg_name, width, spp, seed, scene_seed)
    want, cnt = orc.render(scene, cfg.camera(), params)
    got, st = gpu_render(rt, scene, cfg.camera(), params)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


@pytest.mark.parametrize("w,h", [(1, 1), (1, 5), (5, 1), (9, 7)])
def test_degenerate_image_sizes_match_including_nans(w, h, rt, orc):
    cfg = rt.CONFIGS["C1"]
    scene = rt.Scene.generate(cfg.scene, 1)
    cam = rt.Camera.new(cfg.look_from, cfg.look_at, cfg.view_up, cfg.vfov, w / h, 0.0, 10.0, 0.0, 0.0)
    params = rt.render_params(w, h, 3, 10, background=cfg.background())
    want, _ = orc.render(scene, cam, params)
    got, _ = gpu_render(rt, scene, cam, params)
    np.testing.assert_array_equal(got, want)  # W-1 == 0 divides by zero in renderer.rs:141 on both sides


@pytest.mark.parametrize("depth", [0, 1, 2, 7])
def test_depth_limits(depth, rt, orc):
    cfg, scene, _ = setup(rt, "C3", 24, 2)
    params = rt.render_params(cfg.width, cfg.height, 2, depth, background=cfg.background())
    want, _ = orc.render(scene, cfg.camera(), params)
    got, _ = gpu_render(rt, scene, cfg.camera(), params)
    np.testing.assert_array_equal(got, want)
    if depth == 0:
        assert not got.any()


def test_empty_world_is_background(rt, orc):
    b = rt.SceneBuilder()
    sc = b.finish(rt.HittableList())
    cam = rt.Camera()
    params = rt.render_params(16, 9, 2, 5, background=(0.7, 0.8, 1.0))
    got, st = gpu_render(rt, sc, cam, params)
    want, _ = orc.render(sc, cam, params)
    np.testing.assert_array_equal(got, want)
    assert np.allclose(got, np.float32([0.7, 0.8, 1.0]))


def test_instances_media_and_nested_lists(rt, orc):
    # Translate(RotateY(Translate(...))) chains, a medium inside a RotateY, nested
    # lists and a medium whose boundary is a BVH: shapes no sample scene uses.
    b = rt.SceneBuilder()
    white = b.lambertian_from_color((0.7, 0.7, 0.7))
    glass = b.dielectric(1.3)
    light = b.diffuse_light_from_color((5, 5, 5))
    chk = b.lambertian(b.checker(3.0, b.solid((0.9, 0.1, 0.1)), b.checker_from_color(7.0, (0, 0, 1), (1, 1, 0))))
    inner = rt.HittableList()
    inner.add(b.cube((-1, -1, -1), (1, 1, 1), white))
    inner.add(b.sphere((0, 2, 0), 0.7, glass))
    tri = b.tri((-3, 0, -3), (3, 0, -3), (0, 3, -3), chk)
    lst = rt.HittableList()
    lst.add(b.translate(b.rotate_y(b.translate(b.list(inner), (0.5, 0, 0)), 33.0), (0, 0, 1)))
    lst.add(tri)
    spheres = rt.HittableList()
    for i in range(9):
        spheres.add(b.sphere((i - 4.0, -1.5, 0.5 * (i % 3)), 0.4, white))
    fog_boundary = b.bvh(spheres, 0.0, 1.0, axis_seed=77)
    w = rt.HittableList()
    w.add(b.list(lst))
    w.add(b.rotate_y(b.constant_medium_from_color(b.cube((-2, -2, -2), (2, 2, 2), white), 0.3, (0.2, 0.9, 0.3)), 10.0))
    w.add(b.constant_medium(fog_boundary, 2.0, b.solid((0.9, 0.9, 0.9))))
    w.add(b.xy_rect(-5, 5, 3, 6, -6, light))
    w.add(b.moving_sphere((2, 1, 2), (3, 2, 2), 0.0, 1.0, 0.5, b.metal((0.9, 0.8, 0.7), 0.3)))
    sc = b.finish(w)
    cam = rt.Camera.new((0, 3, 12), (0, 0, 0), (0, 1, 0), 40.0, 1.5, 0.2, 12.0, 0.0, 1.0)
    for exact in (False, True):
        params = rt.render_params(30, 20, 4, 20, background=(0.5, 0.6, 0.7), exact_bvh=exact)
        want, _ = orc.render(sc, cam, params)
        got, _ = gpu_render(rt, sc, cam, params)
        np.testing.assert_array_equal(got, want)


def _mesh_scene(rt):
    # Triangle-BVH scene (the kFSusp preset: the suspending list walk): a lat-long sphere
    # mesh of 1,152 triangles in a BVH under RotateY + Translate, a second BVH (spheres),
    # a fog medium with a sphere boundary between them (its ln(U) draw must stay in list
    # order when a lane's walk is suspended), glass, a light and a ground sphere.
    b = rt.SceneBuilder()
    white = b.lambertian_from_color((0.73, 0.73, 0.73))
    red = b.lambertian_from_color((0.65, 0.05, 0.05))
    glass = b.dielectric(1.5)
    light = b.diffuse_light_from_color((6, 6, 6))
    nu, nv = 32, 18
    tris = rt.HittableList()
    for j in range(nv):
        for i in range(nu):
            pts = []
            for (a, c) in ((i, j), (i + 1, j), (i + 1, j + 1), (i, j + 1)):
                th, ph = np.pi * c / nv, 2 * np.pi * a / nu
                pts.append((1.5 * np.sin(th) * np.cos(ph), 1.5 * np.cos(th), 1.5 * np.sin(th) * np.sin(ph)))
            tris.add(b.tri(pts[0], pts[1], pts[2], red if (i + j) % 5 == 0 else white))
            tris.add(b.tri(pts[0], pts[2], pts[3], white))
    balls = rt.HittableList()
    for i in range(24):
        balls.add(b.sphere((0.9 * (i % 6) - 2.5, 0.4 + 0.5 * (i // 6), -2.0 - 0.3 * (i % 2)), 0.3, white))
    w = rt.HittableList()
    w.add(b.sphere((0, -1000.5, 0), 1000.0, white))
    w.add(b.bvh(balls, 0.0, 1.0, axis_seed=3))
    w.add(b.constant_medium_from_color(b.sphere((0, 1, 0), 4.5, glass), 0.05, (0.9, 0.9, 0.95)))
    w.add(b.translate(b.rotate_y(b.bvh(tris, 0.0, 1.0, axis_seed=11), 20.0), (0.3, 1.2, 0.5)))
    w.add(b.sphere((2.3, 0.5, 1.5), 0.5, glass))
    w.add(b.xz_rect(-2, 2, -2, 2, 5.5, light))
    return b.finish(w)


@pytest.mark.parametrize("w,h,spp", [(64, 48, 6), (9, 1, 4)])
def test_suspending_walk_matches_oracle(w, h, spp, rt, orc):
    # The triangle-BVH preset suspends the long tails of BVH traversals and resumes them on a
    # later trip of the sample loop (kernel.hip world_walk): same bits and segment counts as
    # the oracle, also for H = 1 (every ray has an infinite 1/d and goes to the reference kernel).
    sc = _mesh_scene(rt)
    cam = rt.Camera.new((0, 2, 9), (0, 1, 0), (0, 1, 0), 40.0, w / h, 0.05, 9.0, 0.0, 1.0)
    params = rt.render_params(w, h, spp, 16, background=(0.05, 0.05, 0.08), seed=7)
    want, cnt = orc.render(sc, cam, params)
    got, st = gpu_render(rt, sc, cam, params)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


def _planar_basis(rt, case):
    """A constructed Camera (src/camera.rs:6-27's nine fields) whose every camera ray has an
    exactly zero direction component: origin and lower-left corner share that coordinate,
    horizontal and vertical have none, no lens. "zero_dx": the rays fan in the plane x = 278
    through C4's Cornell box and mesh (cornell_boundaries + the mesh at (325, 0, 200),
    src/main.rs:688-743, 791-802). "nan_closest": they fan in the back wall's plane z = 555, so
    the back wall (xy_rect k = 555, the last rect before the mesh) gives every camera ray
    (k - o) / d = 0 / 0 = NaN, which rectangle.rs:36-65 accepts whatever closest_so_far was."""
    if case == "zero_dx":
        return rt.CameraBasis(origin=(278.0, 278.0, -800.0), horizontal=(0.0, 0.0, 700.0),
                              vertical=(0.0, 556.0, 0.0), lower_left_corner=(278.0, 0.0, 0.0),
                              u=(0.0, 0.0, 1.0), v=(0.0, 1.0, 0.0), lens_radius=0.0, time_start=0.0, time_end=0.0)
    return rt.CameraBasis(origin=(278.0, 278.0, 555.0), horizontal=(556.0, 0.0, 0.0),
                          vertical=(0.0, 556.0, 0.0), lower_left_corner=(0.0, 0.0, 555.0),
                          u=(1.0, 0.0, 0.0), v=(0.0, 1.0, 0.0), lens_radius=0.0, time_start=0.0, time_end=0.0)


@pytest.mark.parametrize("case", ["zero_dx", "nan_closest"])
@pytest.mark.parametrize("suspend", [True, False])
def test_zero_direction_component_on_the_triangle_bvh(case, suspend, rt, orc, capfd):
    # Since round 6 the fast traversal takes rays with a zero direction component into a
    # triangle-only BVH (kernel.hip ray_route, in the fast kernel and the replay pass): 1/d = inf,
    # and the only NaN slab values, 0 * inf on a plane through the origin, are ignored by max / min
    # exactly as aabb.rs:28-41's comparisons ignore them. "zero_dx": every camera ray has d.x == 0
    # and crosses the mesh; the fast kernel traces every sample itself (none is handed over).
    # "nan_closest": every camera ray takes the back wall's 0 / 0 = NaN hit, so the mesh BVH is
    # entered with a NaN closest_so_far (every reference box test passes then): the replay pass
    # takes the literal recursion. Both match the oracle bit for bit, segment counts included,
    # through the suspending walk (the product's triangle preset) and through the all-features
    # instance (`suspend` False: the scene gets a sphere run).
    cfg = rt.CONFIGS["C4"]
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed) if suspend else _c4_with_spheres(rt)
    basis = _planar_basis(rt, case)
    params = rt.render_params(48, 36, 3, 8, background=cfg.background(), seed=3)
    want, cnt = orc.render(scene, basis, params)
    capfd.readouterr()
    with rt.options(launch_log=1):
        got, st = gpu_render(rt, scene, basis, params)
    err = capfd.readouterr().err
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]
    replayed = sum(int(x.split("chunk")[1].split(":")[1].split()[0]) for x in err.splitlines()
                   if "samples replayed" in x)
    assert replayed == (0 if case == "zero_dx" else 48 * 36 * 3), (replayed, err[-2000:])


@pytest.mark.parametrize("suspend", [True, False])
def test_nan_closest_rays_that_hit_the_triangle_bvh(suspend, rt, orc, capfd):
    # A triangle-only BVH entered with a NaN closest_so_far, where the rays do hit triangles (the
    # "nan_closest" case above only has rays that miss the mesh): an xy_rect at z = 200 first in the
    # list gives every camera ray of a fan in the plane z = 200 the hit (k - o) / d = 0 / 0 = NaN
    # (rectangle.rs:36-65 accepts it), then the mesh BVH, whose triangles straddle that plane. The
    # fast kernel hands every sample over; the replay pass takes kernel.hip bvh_hit_nan_tmax (the
    # leaf scan in DFS order up to the first hit, then the fast traversal) instead of the literal
    # recursion. Bits and segment counts must be the oracle's; `suspend` False adds a sphere run
    # (the all-features instance).
    b = rt.SceneBuilder()
    white = b.lambertian_from_color((0.73, 0.73, 0.73))
    red = b.lambertian_from_color((0.65, 0.05, 0.05))
    light = b.diffuse_light_from_color((15.0, 15.0, 15.0))
    w = rt.HittableList()
    w.add(b.xy_rect(0, 555, 0, 555, 200, white))
    w.add(b.xz_rect(213, 343, 227, 332, 554, light))
    mesh = rt.HittableList()
    rng = np.random.default_rng(5)
    for _ in range(400):
        c = rng.uniform((120, 40, 170), (440, 520, 230))
        e = rng.uniform(-45, 45, size=(2, 3))
        mesh.add(b.tri(tuple(c), tuple(c + e[0]), tuple(c + e[1]), red if rng.uniform() < 0.5 else white))
    w.add(b.bvh(mesh, 0.0, 1.0, axis_seed=9))
    w.add(b.xz_rect(0, 555, 0, 555, 0, white))
    if not suspend:
        for i in range(10):
            w.add(b.sphere((1000.0 + 10 * i, 2000.0, 3000.0), 1.0, white))
    scene = b.finish(w)
    basis = rt.CameraBasis(origin=(278.0, 278.0, 200.0), horizontal=(556.0, 0.0, 0.0), vertical=(0.0, 556.0, 0.0),
                           lower_left_corner=(0.0, 0.0, 200.0), u=(1.0, 0.0, 0.0), v=(0.0, 1.0, 0.0),
                           lens_radius=0.0, time_start=0.0, time_end=0.0)
    params = rt.render_params(40, 30, 3, 8, background=(0.05, 0.05, 0.08), seed=13)
    want, cnt = orc.render(scene, basis, params)
    assert np.isfinite(want).all() and (want > 0).any()
    capfd.readouterr()
    with rt.options(launch_log=1):
        got, st = gpu_render(rt, scene, basis, params)
    err = capfd.readouterr().err
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]
    replayed = sum(int(x.split("chunk")[1].split(":")[1].split()[0]) for x in err.splitlines()
                   if "samples replayed" in x)
    assert replayed == 40 * 30 * 3, (replayed, err[-2000:])


def _c4_with_spheres(rt):
    """cornell_boundaries + a triangle mesh BVH (a tetrahedral fan around (325, 100, 200)) + a
    top-level sphere run, built through SceneBuilder so that the scene has spheres and
    triangles (the all-features instance)."""
    b = rt.SceneBuilder()
    red = b.lambertian_from_color((0.65, 0.05, 0.05))
    white = b.lambertian_from_color((0.73, 0.73, 0.73))
    green = b.lambertian_from_color((0.12, 0.45, 0.15))
    light = b.diffuse_light_from_color((15.0, 15.0, 15.0))
    w = rt.HittableList()
    w.add(b.yz_rect(0, 555, 0, 555, 555, green))
    w.add(b.yz_rect(0, 555, 0, 555, 0, red))
    w.add(b.xz_rect(213, 343, 227, 332, 554, light))
    w.add(b.xz_rect(0, 555, 0, 555, 0, white))
    w.add(b.xz_rect(0, 555, 0, 555, 555, white))
    w.add(b.xy_rect(0, 555, 0, 555, 555, white))
    mesh = rt.HittableList()
    rng = np.random.default_rng(11)
    for _ in range(300):
        c = rng.uniform((180, 20, 60), (470, 300, 340))
        e = rng.uniform(-40, 40, size=(2, 3))
        mesh.add(b.tri(tuple(c), tuple(c + e[0]), tuple(c + e[1]), white))
    w.add(b.translate(b.bvh(mesh, 0.0, 1.0, axis_seed=4), (0.0, 0.0, 0.0)))
    for i in range(10):
        w.add(b.sphere((1000.0 + 10 * i, 2000.0, 3000.0), 1.0, white))
    return b.finish(w)


@pytest.mark.parametrize("cfg_name,width,spp", [("C1", 64, 4), ("C3", 48, 3), ("C4", 40, 2)])
def test_bvh_shapes_render_the_same_bits(cfg_name, width, spp, rt, orc):
    # The fast kernel's BVH4 is rebuilt by SAH over the reference tree's leaf nodes (the default,
    # RT_OPT_BVH_SHAPE 0) or collapsed from the reference tree as built (1): different trees, the
    # same visit set of leaf nodes and the same (t, DFS rank) winner, so the same bits and segments.
    cfg, scene, params = setup(rt, cfg_name, width, spp)
    want, cnt = orc.render(scene, cfg.camera(), params)
    for shape in (0, 1):
        with rt.options(bvh_shape=shape):
            got, st = gpu_render(rt, scene, cfg.camera(), params)
        np.testing.assert_array_equal(got, want)
        assert st["segments"] == cnt["segments"]


# --- sharding / determinism (the multi-GPU decomposition) ---------------------------
@pytest.mark.parametrize("n", [2, 3, 8])
def test_gpu_shards_compose_bit_identically(n, rt):
    cfg, scene, params = setup(rt, "C3", 64, 3)
    ds = rt.DeviceScene(scene)
    full, _ = ds.render(cfg.camera(), params)
    acc = np.zeros_like(full)
    for k in range(n):
        p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                             shard_index=k, shard_count=n)
        ds.render(cfg.camera(), p, out=acc)
    ds.close()
    np.testing.assert_array_equal(acc, full)


@pytest.mark.parametrize("n", [1, 3])
def test_block_order_does_not_change_the_image(n, rt, orc):
    # The fast kernel takes a shard's blocks last first (bottom rows first: a short drain);
    # RT_OPT_TUNE bit 21 restores the top-first order. Samples are keyed by pixel and global
    # index and resolved per slot in sample order, so both orders give the oracle's bits, for
    # the whole frame and for a shard (a ragged 61 x 35 image: partial blocks at both edges).
    cfg, scene, params = setup(rt, "C3", 61, 3)
    want, cnt = orc.render(scene, cfg.camera(), params)
    for tune in (0, 1 << 21):
        with rt.options(tune=tune):
            ds = rt.DeviceScene(scene)
            try:
                acc = np.zeros_like(want)
                segs = 0
                for k in range(n):
                    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                                         seed=1, shard_index=k, shard_count=n)
                    _, st = ds.render(cfg.camera(), p, out=acc)
                    segs += st["segments"]
            finally:
                ds.close()
        np.testing.assert_array_equal(acc, want)
        assert segs == cnt["segments"]


def test_repeat_renders_are_bit_identical(rt):
    cfg, scene, params = setup(rt, "C5", 64, 4)
    ds = rt.DeviceScene(scene)
    a, _ = ds.render(cfg.camera(), params)
    b, _ = ds.render(cfg.camera(), params)
    ds.close()
    np.testing.assert_array_equal(a, b)


# --- full BASELINE sizes --------------------------------------------------------------
def test_c3_full_resolution_one_spp_matches_oracle(rt, orc):
    cfg, scene, params = setup(rt, "C3", 1200, 1)
    assert (cfg.width, cfg.height) == (1200, 800)
    want, _ = orc.render(scene, cfg.camera(), params)
    got, _ = gpu_render(rt, scene, cfg.camera(), params)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("cfg_name,shard", [("C2", 137), ("C3", 101), ("C4", 77), ("C5", 200)])
def test_full_workload_subsample_matches_oracle(cfg_name, shard, rt, orc):
    # the full-size render on the GPU (C2 1200x800x500 over the 485-sphere list with the f32
    # pretest, C3 1200x800x500, C4 1920x1080x1000 over the 20k-triangle mesh, C5 1920x1080x2000
    # with the media), checked bit-exactly on a
    # 1/256 block shard rendered by the oracle at the same full spp and depth
    cfg = rt.CONFIGS[cfg_name]
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    params = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background())
    got, st = gpu_render(rt, scene, cfg.camera(), params)
    assert st["samples"] == cfg.width * cfg.height * cfg.spp
    sub = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                           shard_index=shard, shard_count=256)
    want = np.full_like(got, np.nan)
    _, cnt = orc.render(scene, cfg.camera(), sub, out=want)
    mask = ~np.isnan(want[..., 0])
    assert mask.sum() > 3000
    np.testing.assert_array_equal(got[mask], want[mask])
    assert np.isfinite(got).all()
    # the same shard rendered alone on the GPU: its pixels and its segment count (a draw-count
    # drift that left the shard's pixels unchanged would still move the count)
    shard, st_sh = gpu_render(rt, scene, cfg.camera(), sub)
    np.testing.assert_array_equal(shard[mask], want[mask])
    assert st_sh["samples"] == int(mask.sum()) * cfg.spp
    assert st_sh["segments"] == cnt["segments"], (st_sh["segments"], cnt["segments"])


def test_c1_full_frame_matches_oracle(rt, orc):
    # BASELINE config 1 (random_spheres 400x225, 50 spp, depth 50) in full: every pixel and
    # the segment count against the oracle's whole frame (4.5 M samples, a few seconds of CPU)
    import os
    cfg = rt.CONFIGS["C1"]
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    params = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background())
    got, st = gpu_render(rt, scene, cfg.camera(), params)
    want, cnt = orc.render(scene, cfg.camera(), params, threads=max(1, min(16, len(os.sched_getaffinity(0)))))
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


@pytest.mark.parametrize("cfg_name,spp", [("C3", 500), ("C2", 8), ("C1", 16), ("C4", 100)])
def test_pruned_traversal_equals_reference_traversal_full_frame(cfg_name, spp, rt):
    # Closest-hit box pruning and leaf-box rejects must not change a single path:
    # same bits AND the same number of ray segments as the reference's unpruned
    # traversal. C3 runs at its full 500 spp: the rare ray parallel to a cube
    # face through the face's plane (the reference's 0/0 = NaN rect hit) shows
    # up a few dozen times per frame and must be traversed unpruned.
    cfg = rt.CONFIGS[cfg_name]
    cfg = cfg.scaled(cfg.width, spp)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    ds = rt.DeviceScene(scene)
    out = {}
    for exact in (True, False):
        p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(), exact_bvh=exact)
        out[exact] = ds.render(cfg.camera(), p)
    ds.close()
    np.testing.assert_array_equal(out[True][0], out[False][0])
    assert out[True][1]["segments"] == out[False][1]["segments"]


@pytest.mark.parametrize("cfg_name,spp", [("C1", 50), ("C3", 500), ("C4", 100)])
def test_traversal_audit_full_frame(cfg_name, spp):
    # The audit build replays EVERY fast BVH traversal of a full C1 frame, a full C3 frame
    # (500 spp) and a full-resolution C4 frame (the suspending walk over the triangle BVH)
    # with the literal bvh.rs recursion and re-tests every leaf-box reject; both counts
    # must be 0. The bounds count also covers take_sample's invariant that the whole wave
    # is active where lane 0 claims a batch (kernel.hip take_sample).
    # Per-call (t, primitive) equality is stricter than the image tests: a tie resolved
    # to the wrong coplanar face can shade identically.
    import subprocess
    import sys
    root = os.path.dirname(HERE)
    lib = os.path.join(root, "raytracinginoneweekendinrust_amd", "_lib", "librtamd_audit.so")
    assert os.path.exists(lib), "build() makes the audit library"
    env = dict(os.environ, RT_LIBRARY=lib)
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "region_profile.py"), "--config", cfg_name,
                        "--spp", str(spp)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout + r.stderr
    assert '{"leaf_audit_count": 0}' in out, out[-2000:]
    assert '{"trav_audit_count": 0}' in out, out[-2000:]
    assert '{"bounds_audit_count": 0}' in out, out[-2000:]  # every visited node index and stack slot in range


def test_sphere_pretest_audit_c2():
    # C2's 485-sphere list takes the f32 discriminant pretest; the audit build
    # re-runs the f64 test on every pretest reject and counts any it would accept.
    import subprocess
    import sys
    root = os.path.dirname(HERE)
    lib = os.path.join(root, "raytracinginoneweekendinrust_amd", "_lib", "librtamd_audit.so")
    env = dict(os.environ, RT_LIBRARY=lib)
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "region_profile.py"), "--config", "C2",
                        "--spp", "16"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout + r.stderr
    assert '{"leaf_audit_count": 0}' in out, out[-2000:]


@pytest.mark.parametrize("with_tri", [False, True])
def test_every_feature_preset_instance(with_tri, rt, orc):
    # A long top-level sphere run (the f32 pretest), a BVH and, optionally, a
    # triangle: the scene needs the all-features instance of the fast kernel
    # (the flat / BVH-only presets are exercised by the C1-C5 cases above).
    b = rt.SceneBuilder()
    white = b.lambertian_from_color((0.7, 0.7, 0.7))
    metal = b.metal((0.8, 0.6, 0.2), 0.1)
    w = rt.HittableList()
    for i in range(11):
        w.add(b.sphere((i - 5.0, 0.3 * (i % 3), -1.0 - 0.2 * (i % 2)), 0.45, metal if i % 2 else white))
    inner = rt.HittableList()
    for i in range(12):
        inner.add(b.sphere((i - 6.0, 1.6, 0.5 * (i % 4)), 0.35, white))
    w.add(b.bvh(inner, 0.0, 1.0, axis_seed=5))
    if with_tri:
        w.add(b.tri((-6, -1, -3), (6, -1, -3), (0, 4, -3), white))
    w.add(b.sphere((0, -1000.5, 0), 1000.0, white))
    sc = b.finish(w)
    cam = rt.Camera.new((0, 2, 9), (0, 0.5, 0), (0, 1, 0), 45.0, 1.5, 0.05, 9.0, 0.0, 0.0)
    params = rt.render_params(36, 24, 4, 12, background=(0.6, 0.7, 0.9))
    want, cnt = orc.render(sc, cam, params)
    got, st = gpu_render(rt, sc, cam, params)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


@pytest.mark.parametrize("cfg_name", ["C3", "C4"])
def test_stack_spill_to_hbm_matches_oracle(cfg_name, rt, orc):
    # Deep BVHs keep kStackLdsMax stack entries in LDS and the rest in HBM; a 2-entry
    # LDS part (rt_set_option(RT_OPT_STACK_LDS), read at upload) sends almost every traversal through
    # the HBM half, on the pruned (C3) and the unpruned triangle (C4) traversal.
    cfg, scene, params = setup(rt, cfg_name, 40, 2, seed=3)
    want, cnt = orc.render(scene, cfg.camera(), params)
    with rt.options(stack_lds=2):
        got, st = gpu_render(rt, scene, cfg.camera(), params)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


@pytest.mark.parametrize("replay_ref", [False, True])
@pytest.mark.parametrize("cfg_name,w,h", [("C3", 40, None), ("C5", 41, None), ("C3", 7, 1)])
def test_replay_pass_kernels_match_oracle(cfg_name, w, h, replay_ref, rt, orc):
    # Samples the fast kernel hands over (rays with a zero / non-finite 1/d component) are
    # re-traced by trace_samples<3> (fast traversal except for those rays), or with
    # RT_OPT_TUNE bit 16 by the literal replay trace_samples<1>. H = 1 makes every ray such a ray.
    cfg, scene, params = setup(rt, cfg_name, w, 3, seed=5)
    cam = cfg.camera()
    if h is not None:
        cam = rt.Camera.new(cfg.look_from, cfg.look_at, cfg.view_up, cfg.vfov, w / h, cfg.aperture,
                            cfg.focus_dist, cfg.time0, cfg.time1)
        params = rt.render_params(w, h, 3, cfg.depth, background=cfg.background(), seed=5)
    want, cnt = orc.render(scene, cam, params)
    with rt.options(tune=(1 << 16) if replay_ref else 0):
        got, st = gpu_render(rt, scene, cam, params)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


@pytest.mark.parametrize("stream", [True, False, "frames_in_flight"])
@pytest.mark.parametrize("cfg_name", ["C3", "C5", "C4"])
def test_streaming_replay_pass_matches_oracle(cfg_name, stream, rt, orc):
    # The streaming replay pass (kernel.hip replay_claim) runs beside the fast kernel and takes
    # the handed-over samples while the fast kernel drains; RT_OPT_TUNE bit 17 leaves them all
    # to the serialized pass, and so does the public RT_FLAG_FRAMES_IN_FLIGHT (bench.py's N > 1 step). A 4096 x 1 image (v = j / (H - 1) = NaN: every ray is handed
    # over) with 8 spp gives 4096 work units, enough to fill the GPU, so the fast kernel's
    # waves drain while the stream's waves wait for slots, and every sample is replayed.
    # C4 is the deep-stack case: its replay runs trace_samples<3, 3, kFAll> and the streaming
    # waves spill into their own slabs behind the fast kernel's (the grid + kStreamWaves layout).
    cfg = rt.CONFIGS[cfg_name]
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    w, h, spp = 4096, 1, 8
    cam = rt.Camera.new(cfg.look_from, cfg.look_at, cfg.view_up, cfg.vfov, w / h, cfg.aperture, cfg.focus_dist,
                        cfg.time0, cfg.time1)
    params = rt.render_params(w, h, spp, cfg.depth, background=cfg.background(), seed=9)
    want, cnt = orc.render(scene, cam, params)
    if stream == "frames_in_flight":
        params = rt.render_params(w, h, spp, cfg.depth, background=cfg.background(), seed=9, frames_in_flight=True)
    with rt.options(tune=1 << 17 if stream is False else 0):
        ds = rt.DeviceScene(scene)
        try:
            for _ in range(2):  # the second render starts from the list the first one freed
                got, st = ds.render(cam, params)
                np.testing.assert_array_equal(got, want)
                assert st["segments"] == cnt["segments"]
        finally:
            ds.close()


def test_medium_first_fallback_stays_exact():
    # The medium-first bound walks the entries before the first medium with a bound
    # from an f32 estimate of the scatter point, and hands the sample to the reference kernel when
    # the exact values contradict the estimate. That fallback is rare with the real estimate; the
    # audit build's RT_OPT_TUNE kModeMbShrink (bit 29) halves the estimate so that it fires on
    # most segments inside the dense medium. A 1/256 C3 shard at 64 spp must still match the
    # oracle bit for bit, and the launch log must show many more hand-overs than without it.
    import subprocess
    import sys
    root = os.path.dirname(HERE)
    lib = os.path.join(root, "raytracinginoneweekendinrust_amd", "_lib", "librtamd_audit.so")
    assert os.path.exists(lib), "build() makes the audit library"
    code = r'''
import sys, json, numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {oracle!r})
import raytracinginoneweekendinrust_amd as rt, oracle_ffi as orc
cfg = rt.CONFIGS["C3"]
scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
p = rt.render_params(cfg.width, cfg.height, 64, cfg.depth, background=cfg.background(), shard_index=101, shard_count=256)
want = np.full(cfg.width * cfg.height * 3, np.nan, dtype=np.float32)
_, cnt = orc.render(scene, cfg.camera(), p, out=want, threads=8)
ds = rt.DeviceScene(scene)
got, st = ds.render(cfg.camera(), p)
ds.close()
got = np.asarray(got).reshape(-1)
m = ~np.isnan(want)
print(json.dumps({{"equal": bool((got[m] == want[m]).all()), "segments": int(st["segments"]), "oracle": int(cnt["segments"])}}))
'''.format(root=root, oracle=os.path.join(root, "oracle"))
    counts = {}
    for tune in ("0", str(1 << 29)):
        env = dict(os.environ, RT_LIBRARY=lib)
        r = subprocess.run([sys.executable, "-c", "import os, raytracinginoneweekendinrust_amd as rt\n"
                            f"rt.set_option('tune', {tune}); rt.set_option('launch_log', 1)\n" + code],
                           capture_output=True, text=True, env=env, timeout=600, cwd=root)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
        assert res["equal"], (tune, res)
        assert res["segments"] == res["oracle"], (tune, res)
        counts[tune] = sum(int(x.split("chunk")[1].split(":")[1].split()[0]) for x in r.stderr.splitlines()
                           if "samples replayed" in x)
    assert counts[str(1 << 29)] > 10 * max(counts["0"], 1), counts
