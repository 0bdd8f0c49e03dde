"""The drop-in boundary on the device: caller-built Bvh trees (RT_OBJ_BVH_TREE,
src/bvh.rs:38-43), a constructed Camera (rt_camera, src/camera.rs:6-27), OBJ
ingestion with tobj's models[0] (src/main.rs:745-789), progressive multi-device
frames, per-handle launch serialisation and the multi-process shard gather.
Bar: bit-exact against the oracle / the one-device render."""
import threading

import numpy as np
import pytest

from tree_util import sphere_scene

pytestmark = pytest.mark.gpu


def _cam(rt):
    return rt.Camera((13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, 1.5, 0.1, 10.0, 0.0, 1.0)


@pytest.mark.parametrize("tree", ["random", "median-x"])
def test_prebuilt_tree_and_camera_basis_match_oracle(rt, orc, tree):
    scene = sphere_scene(rt, n=150, seed=11, tree=tree)
    basis = rt.CameraBasis.from_camera(_cam(rt))
    basis.lens_radius = 0.07            # a Camera no Camera::new call with these arguments makes
    basis.vertical = tuple(np.float32(x) * np.float32(1.01) for x in basis.vertical)
    p = rt.render_params(72, 48, 8, 12, background=(0.7, 0.8, 1.0))
    ds = rt.DeviceScene(scene)
    try:
        got, st = ds.render(basis, p)
    finally:
        ds.close()
    want, cnt = orc.render(scene, basis, p)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


def test_prebuilt_tree_with_moving_spheres_ignores_tree_times(rt, orc):
    """A caller's Bvh stores no shutter times (bvh.rs:38-43): a tree of spheres, cubes and
    moving spheres handed over with f[0] = f[1] = 0 renders exactly like the oracle, which
    tests only the caller's node boxes (leaf rejects must not use those times)."""
    scene = sphere_scene(rt, n=60, seed=23, tree="median-x", moving=40, tree_times=(0.0, 0.0))
    p = rt.render_params(64, 40, 8, 10, background=(0.7, 0.8, 1.0))
    ds = rt.DeviceScene(scene)
    try:
        got, st = ds.render(_cam(rt), p)
    finally:
        ds.close()
    want, cnt = orc.render(scene, _cam(rt), p)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


def test_prebuilt_tree_with_boxes_smaller_than_their_objects(rt, orc):
    """A caller's leaf boxes need not contain their objects (the reference tests only the
    boxes, bvh.rs:363-417): a sphere sticking out of its box toward the ray can be hit
    before that box is entered, so such a tree is lowered without closest-hit pruning."""
    scene = sphere_scene(rt, n=150, seed=31, tree="median-x", box_scale=0.6)
    p = rt.render_params(72, 48, 8, 12, background=(0.7, 0.8, 1.0))
    ds = rt.DeviceScene(scene)
    try:
        got, st = ds.render(_cam(rt), p)
    finally:
        ds.close()
    want, cnt = orc.render(scene, _cam(rt), p)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


def test_camera_basis_equals_camera_new_on_device(rt):
    cfg = rt.CONFIGS["C3"].scaled(48, 4)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background())
    ds = rt.DeviceScene(scene)
    try:
        a, sa = ds.render(cfg.camera(), p)
        b, sb = ds.render(rt.CameraBasis.from_camera(cfg.camera()), p)
    finally:
        ds.close()
    np.testing.assert_array_equal(a, b)
    assert sa["segments"] == sb["segments"]


OCTA_AND_JUNK = (
    "o octahedron\n"
    "v 0 160 0\nv 150 0 0\nv 0 0 150\nv -150 0 0\nv 0 0 -150\nv 0 -160 0\n"
    "f 1 3 2\nf 1 4 3\nf 1 5 4\nf 1 2 5\nf 6 2 3 \nf 6/1/1 3/1/1 4/1/1\nf 6 4 5\nf -1 -5 -4\n"
    "o junk\nv 0 0 0\nv 500 0 0\nv 0 500 0\nf 7 8 9\n")


def test_obj_models0_bunny_matches_oracle(rt, orc, tmp_path):
    (tmp_path / "bunny_2000_scale.obj").write_text(OCTA_AND_JUNK)
    (tmp_path / "earthmap_1024x512.rgb8").write_bytes(b"")
    scene = rt.Scene.generate("bunny", 1, str(tmp_path))
    n = scene.nodes()
    assert (n["kind"] == 38).sum() == 8  # the octahedron only (models[0])
    cfg = rt.CONFIGS["C4"].scaled(48, 4)
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background())
    ds = rt.DeviceScene(scene)
    try:
        got, st = ds.render(cfg.camera(), p)
    finally:
        ds.close()
    want, cnt = orc.render(scene, cfg.camera(), p)
    np.testing.assert_array_equal(got, want)
    assert st["segments"] == cnt["segments"]


def test_render_multi_progressive_accumulate_equals_one_shot(rt):
    cfg = rt.CONFIGS["C3"].scaled(40, 6)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background())
    hs = [rt.DeviceScene(scene, 0), rt.DeviceScene(scene, 0)]
    try:
        one, _ = hs[0].render(cfg.camera(), p)
        acc = np.zeros_like(one)
        done = 0
        for n in (2, 1, 3):
            q = rt._capi.rt_render_params.from_buffer_copy(p)
            q.sample_base, q.samples_per_pixel = done, n
            last = done + n == cfg.spp
            q.flags = (rt._capi.RT_FLAG_ACCUMULATE if done else 0) | (0 if last else rt._capi.RT_FLAG_RAW_SUM)
            q.spp_total = cfg.spp if last else 0
            rt.render_multi(hs, cfg.camera(), q, out=acc)
            done += n
    finally:
        for h in hs:
            h.close()
    np.testing.assert_array_equal(acc, one)


def test_concurrent_renders_on_one_handle_are_serialised(rt):
    cfg = rt.CONFIGS["C3"].scaled(40, 4)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    ds = rt.DeviceScene(scene)
    params = [rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(), seed=s)
              for s in (1, 2, 3, 4)]
    try:
        serial = [ds.render(cfg.camera(), q)[0] for q in params]
        out = [None] * len(params)

        def work(i):
            for _ in range(3):
                out[i] = ds.render(cfg.camera(), params[i])[0]

        th = [threading.Thread(target=work, args=(i,)) for i in range(len(params))]
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        ds.close()
    for a, b in zip(out, serial):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("w,h", [(1200, 800), (37, 29), (8, 8)])
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_shard_pack_unpack_round_trip(rt, w, h, n):
    import torch
    g = torch.Generator(device="cuda").manual_seed(w * 31 + n)
    img = torch.rand(w * h * 3, device="cuda", generator=g)
    total = rt.shard_offset(w, h, n, n)
    packed = torch.full((total,), float("nan"), device="cuda")
    for r in range(n):
        # each rank renders only its blocks: the rest of its image is garbage it must not ship
        mine = torch.where(rt.shard_mask(w, h, r, n, device="cuda").repeat_interleave(3), img, torch.full_like(img, -7.0))
        off, cnt = rt.shard_offset(w, h, r, n), rt.shard_floats(w, h, r, n)
        rt.shard_pack(mine, w, h, r, n, packed[off: off + cnt])
    out = torch.zeros_like(img)
    rt.shard_unpack(packed, w, h, n, out)
    torch.cuda.synchronize()
    assert torch.equal(out, img)
