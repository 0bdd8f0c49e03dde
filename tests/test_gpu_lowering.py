"""Lowering structure on the device (rt_scene_info): the run entries of round 5.

Consecutive untransformed top-level rectangles with consecutive records lower into one
kEntRectRun entry walked in list order (csrc/lower.cpp), the same way spheres lower into
sphere runs; the images are covered bit for bit by the parity files. Here: the Cornell
scenes' six walls (the light included) are one entry."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg_name,entries", [("C4", 2), ("C5", 5)])
def test_cornell_walls_lower_to_one_rect_run(cfg_name, entries, rt):
    # C4: the wall run and the mesh BVH; C5: the wall run, the two smoke media and their two
    # Cube boundaries (appended after the top-level entries)
    cfg = rt.CONFIGS[cfg_name]
    ds = rt.DeviceScene(rt.Scene.generate(cfg.scene, cfg.scene_seed))
    try:
        info = ds.info()
    finally:
        ds.close()
    assert info["entries"] == entries, info
    assert info["rects"] >= 6, info
