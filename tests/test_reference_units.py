"""The reference's own unit tests and doc-comment known answers, run against the
oracle restatement and (where the product exposes the function) the product.

src/renderer.rs:311-377  Tile::tile (tile_perfect_tiling, tile_imperfect_tiling)
src/aabb.rs:73-140       Aabb::hit / Aabb::union (6 tests)
src/geometry/sphere.rs:37-40  Sphere::get_uv examples
Random123 kat_vectors    Philox4x32-10 (the RNG that replaces thread_rng)
"""
import math

import numpy as np
import pytest


@pytest.mark.parametrize("which", ["oracle", "product"])
def test_tile_perfect_tiling(which, rt, orc):  # renderer.rs:311-338
    tiles = orc.tile(300, 30, 100, 10) if which == "oracle" else rt.tile(300, 30, 100, 10)
    assert len(tiles) == 9
    assert tiles[0] == (100, 10, 0, 0)
    assert tiles[1] == (100, 10, 100, 0)
    assert tiles[3][2:] == (0, 10)
    assert tiles[-1] == (100, 10, 200, 20)


@pytest.mark.parametrize("which", ["oracle", "product"])
def test_tile_imperfect_tiling(which, rt, orc):  # renderer.rs:340-377
    tiles = orc.tile(310, 31, 100, 10) if which == "oracle" else rt.tile(310, 31, 100, 10)
    assert len(tiles) == 16
    assert tiles[0] == (100, 10, 0, 0)
    assert tiles[4] == (100, 10, 0, 10)
    assert tiles[3] == (10, 10, 300, 0)
    assert tiles[12] == (100, 1, 0, 30)
    assert tiles[15] == (10, 1, 300, 30)


@pytest.mark.parametrize("w,h,tw,th", [(1, 1, 8, 8), (7, 5, 8, 8), (64, 64, 8, 8), (1200, 800, 8, 8),
                                        (1921, 1081, 16, 4), (9, 17, 3, 5)])
def test_tile_oracle_and_product_agree_and_cover(w, h, tw, th, rt, orc):
    a, b = orc.tile(w, h, tw, th), rt.tile(w, h, tw, th)
    assert a == b
    cover = np.zeros((h, w), dtype=np.int32)
    for (tw_, th_, x, y) in a:
        cover[y:y + th_, x:x + tw_] += 1
    assert (cover == 1).all()


def test_tile_rejects_zero_size(rt):
    with pytest.raises(rt.RTError):
        rt.tile(10, 10, 0, 8)


def test_aabb_hits(orc):  # aabb.rs:73-84
    assert orc.aabb_hit((-1, -1, 1), (1, 1, 2), (0, 0, 0), (0, 0, 1), 0.0, 5.0)


def test_aabb_misses(orc):  # aabb.rs:86-97
    assert not orc.aabb_hit((1, 1, 1), (2, 2, 2), (0, 0, 0), (0, 0, 1), 0.0, 5.0)


def test_aabb_union_nones(orc):  # aabb.rs:99-102
    assert orc.aabb_union(None, None) is None


def test_aabb_union_one_side(orc):  # aabb.rs:104-122
    box = (1.0, 1.0, 1.0, 2.0, 2.0, 2.0)
    assert orc.aabb_union(box, None) == box
    assert orc.aabb_union(None, box) == box


def test_aabb_union(orc):  # aabb.rs:124-140
    got = orc.aabb_union((0, 1, 0, 2, 4, 2), (1, 0, 1, 3, 3, 3))
    assert got == (0.0, 0.0, 0.0, 3.0, 4.0, 3.0)


@pytest.mark.parametrize("p,uv", [((1, 0, 0), (0.5, 0.5)), ((-1, 0, 0), (0.0, 0.5)), ((0, 1, 0), (0.5, 1.0)),
                                   ((0, -1, 0), (0.5, 0.0)), ((0, 0, 1), (0.25, 0.5)), ((0, 0, -1), (0.75, 0.5))])
def test_sphere_get_uv_examples(p, uv, orc):  # sphere.rs:37-40
    u, v = orc.sphere_uv(p)
    assert u == pytest.approx(uv[0], abs=1e-6) and v == pytest.approx(uv[1], abs=1e-6)


@pytest.mark.parametrize("ctr,key,expect", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox4x32_10_random123_kat(ctr, key, expect, orc):
    assert tuple(orc.philox(ctr, key)) == expect


def test_camera_basis_book_values(rt, orc):
    # Camera::new for the CLI defaults (src/main.rs:76-96), checked against float64 math
    cam = rt.Camera.new((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 16.0 / 9.0, 0.0, 10.0, 0.0, 0.0)
    b = orc.camera_basis(cam)
    lf = np.array([13, 2, 3.0])
    w = lf / np.linalg.norm(lf)
    u = np.cross([0, 1.0, 0], w)
    u /= np.linalg.norm(u)
    v = np.cross(w, u)
    h = math.tan(math.radians(20.0) / 2)
    hor = 10.0 * (16 / 9 * 2 * h) * u
    ver = 10.0 * (2 * h) * v
    llc = lf - hor / 2 - ver / 2 - 10.0 * w
    np.testing.assert_allclose(b[3:6], hor, rtol=1e-5)
    np.testing.assert_allclose(b[6:9], ver, rtol=1e-5)
    np.testing.assert_allclose(b[9:12], llc, rtol=1e-5)
    assert b[18] == 0.0 and b[19] == 0.0 and b[20] == 0.0


def test_camera_inclusive_time_scale(rt, orc):
    # UniformFloat::new_inclusive(0, 1): scale * max_rand + low <= high (rand 0.8.5)
    cam = rt.Camera.new((0, 0, 0), (0, 0, -1), (0, 1, 0), 40.0, 1.5, 0.0, 10.0, 0.0, 1.0)
    scale = np.float32(orc.camera_basis(cam)[20])
    max_rand = np.float32(1.0) - np.float32(2.0 ** -23)
    assert np.float32(scale * max_rand) <= np.float32(1.0)
    assert scale >= np.float32(1.0)
