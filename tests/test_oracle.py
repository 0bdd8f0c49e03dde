"""CPU oracle self-consistency (no GPU): golden fixtures, integration order,
threading / sharding invariance, libm substitution."""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def golden_cases():
    return json.load(open(os.path.join(GOLDEN, "cases.json")))


@pytest.fixture(scope="module")
def golden():
    return np.load(os.path.join(GOLDEN, "renders.npz"))


@pytest.mark.parametrize("name", sorted(golden_cases()))
def test_oracle_reproduces_golden(name, golden, rt, orc):
    from golden.make_golden import case_setup
    cfg, scene, params = case_setup(rt, golden_cases()[name])
    img, _ = orc.render(scene, cfg.camera(), params)
    np.testing.assert_array_equal(img, golden[name])


def small(rt, cfg_name, width=32, spp=4):
    cfg = rt.CONFIGS[cfg_name].scaled(width, spp)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    params = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background())
    return cfg, scene, params


@pytest.mark.parametrize("cfg_name", ["C1", "C3", "C5"])
def test_forward_product_matches_reference_recursion(cfg_name, rt, orc):
    # src/ray.rs:51-55 evaluates e0 + a0*(e1 + a1*(...)); the device order is the
    # forward product. Same draws and branches, only float reassociation differs.
    cfg, scene, params = small(rt, cfg_name)
    fwd, c1 = orc.render(scene, cfg.camera(), params)
    rec, c2 = orc.render(scene, cfg.camera(), params, flags=orc.FLAG_RECURSIVE)
    assert c1["segments"] == c2["segments"] and c1["node_visits"] == c2["node_visits"]
    np.testing.assert_allclose(fwd, rec, rtol=1e-5, atol=1e-6)


def test_thread_count_does_not_change_bits(rt, orc):
    cfg, scene, params = small(rt, "C3", 40, 3)
    a, _ = orc.render(scene, cfg.camera(), params, threads=1)
    b, _ = orc.render(scene, cfg.camera(), params, threads=7)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_shards_compose_to_full_frame(n, rt, orc):
    cfg, scene, params = small(rt, "C5", 40, 2)
    full, _ = orc.render(scene, cfg.camera(), params)
    acc = np.zeros_like(full)
    for k in range(n):
        p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                             shard_index=k, shard_count=n)
        orc.render(scene, cfg.camera(), p, out=acc)
    np.testing.assert_array_equal(acc, full)


def test_sample_base_splits_the_sample_sequence(rt, orc):
    cfg, scene, _ = small(rt, "C1", 24, 4)
    mk = lambda spp, base: rt.render_params(cfg.width, cfg.height, spp, cfg.depth, background=cfg.background(),
                                            sample_base=base)
    whole, _ = orc.render(scene, cfg.camera(), mk(4, 0))
    a, _ = orc.render(scene, cfg.camera(), mk(2, 0))
    b, _ = orc.render(scene, cfg.camera(), mk(2, 2))
    np.testing.assert_allclose((a + b) / 2, whole, rtol=1e-6, atol=1e-7)


def test_libm_transcendentals_change_almost_nothing(rt, orc):
    # The reference calls glibc through Rust's f32 methods; the spec differs by <= 1 ulp.
    cfg, scene, params = small(rt, "C3", 40, 4)
    spec, _ = orc.render(scene, cfg.camera(), params)
    libm, _ = orc.render(scene, cfg.camera(), params, flags=orc.FLAG_LIBM)
    d = np.abs(np.clip(spec, 0, 1) - np.clip(libm, 0, 1))
    assert (d.max(axis=2) > 1e-3).mean() < 0.02
    assert d.mean() < 1e-3


def test_sample_api_matches_render(rt, orc):
    cfg, scene, params = small(rt, "C1", 16, 1)
    img, _ = orc.render(scene, cfg.camera(), params)
    for (x, y) in [(0, 0), (5, 3), (15, 8)]:
        np.testing.assert_array_equal(orc.sample(scene, cfg.camera(), params, x, y, 0), img[y, x])


def test_depth_zero_is_black_and_depth_one_is_emission_or_background(rt, orc):
    cfg, scene, _ = small(rt, "C1", 16, 2)
    p0 = rt.render_params(cfg.width, cfg.height, 2, 0, background=cfg.background())
    img0, c0 = orc.render(scene, cfg.camera(), p0)
    assert not img0.any() and c0["segments"] == 0
    p1 = rt.render_params(cfg.width, cfg.height, 2, 1, background=cfg.background())
    img1, _ = orc.render(scene, cfg.camera(), p1)
    # a first hit scatters but depth-1 == 0 stops it; only sky pixels are lit
    vals = np.unique(img1.reshape(-1, 3), axis=0)
    assert len(vals) <= 3


def test_invalid_camera_time_range(rt, orc):
    cfg, scene, params = small(rt, "C1", 8, 1)
    cam = rt.Camera.new((13, 2, 3), (0, 0, 0), (0, 1, 0), 20, 1.7, 0, 10, 1.0, 0.0)
    with pytest.raises(RuntimeError):
        orc.render(scene, cam, params)


def _py_bvh_order(keys, seed):
    """BvhNode::new_helper's leaf order (src/bvh.rs:249-333) in plain Python: axis per node
    in preorder from the Philox stream (rand 0.8.5 sample_single_inclusive(0, 2)),
    stable sort by f32 total_cmp (Python's sort is stable), two-item nodes by one compare."""
    import struct
    from oracle_ffi import philox

    def tkey(f):
        u = struct.unpack("<I", struct.pack("<f", f))[0]
        return u ^ (0xFFFFFFFF if u >> 31 else 0x80000000)

    words, block = [], [0]

    def axis():
        while True:
            if not words:
                words.extend(philox([block[0], 0, 0, 0], [seed & 0xFFFFFFFF, seed >> 32]))
                block[0] += 1
            m = words.pop(0) * 3
            if (m & 0xFFFFFFFF) <= (3 << 30) - 1:
                return m >> 32

    def helper(items):
        a = axis()
        if len(items) == 2:
            return items if tkey(keys[items[0]][a]) < tkey(keys[items[1]][a]) else items[::-1]
        if len(items) == 1:
            return items
        items = sorted(items, key=lambda i: tkey(keys[i][a]))
        mid = len(items) // 2
        return helper(items[:mid]) + helper(items[mid:])

    return helper(list(range(len(keys))))


@pytest.mark.parametrize("n,seed", [(1, 3), (2, 3), (3, 1), (9, 20231), (40, 7), (300, 2**33 + 5)])
def test_oracle_bvh_order_matches_python_restatement(n, seed, orc):
    rng = np.random.default_rng(n)
    keys = rng.integers(-2, 3, size=(n, 3)).astype(np.float32)  # many ties
    keys[::5, 0] = -0.0
    got = orc.bvh_order(keys, seed)
    want = _py_bvh_order([tuple(float(x) for x in r) for r in keys], seed)
    assert list(got) == want


def test_prebuilt_tree_oracle_equals_flat_list(rt, orc):
    """RT_OBJ_BVH_TREE in the oracle: a caller-built tree over random spheres and cubes (no
    coincident surfaces, so no ties) gives the flat list's image (hittable.rs:100-118)."""
    from tree_util import sphere_scene
    cam = rt.Camera((13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, 1.5, 0.1, 10.0, 0.0, 1.0)
    p = rt.render_params(36, 24, 4, 8, background=(0.7, 0.8, 1.0))
    a, ca = orc.render(sphere_scene(rt, with_tree=True), cam, p)
    b, cb = orc.render(sphere_scene(rt, with_tree=False), cam, p)
    np.testing.assert_array_equal(a, b)
    assert ca["segments"] == cb["segments"] and ca["node_visits"] > 0 == cb["node_visits"]


def test_camera_basis_oracle_equals_camera_new(rt, orc):
    """oracle_render_camera with Camera::new's fields == oracle_render with its arguments."""
    cfg = rt.CONFIGS["C3"].scaled(32, 2)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background())
    a, _ = orc.render(scene, cfg.camera(), p)
    b, _ = orc.render(scene, rt.CameraBasis.from_camera(cfg.camera()), p)
    np.testing.assert_array_equal(a, b)
