"""The EXEC-join miscompile on hardware (tests/test_exec_join.py is the CPU guard).

librtamd_rngdiv.so is kernel.hip with the per-lane branch around the out-of-line Philox call
(RT_RNG_UNIFORM=0); tools/exec_join_check.py finds the Rng buffer's two split copies ahead of
that join's EXEC restore (in round 4 in its C1 and C4 instances; since round 5's DevScene grew by
a word, in the all-features instance, which the second case renders). Here the fixture renders
one sample index of C1: the camera segment (depth 1) still matches the oracle, the full path does not, first at
pixel (3, 0), whose lane entered its first scatter with r0 = d (tools/trace_sample.py recorded
r0 = 6, r2 = a stale float, d = 7 on this box). The product renders the same sample bit-exact.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "_lib")


def test_fixture_leaves_the_oracle_after_the_camera_segment_only(rt, orc):
    # (the name is round 4's, when the split sat after C1's camera segment; which segment goes
    # wrong first depends on where the split join is, so only "the fixture leaves the oracle and
    # the product does not" is asserted)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from ab_time import bind
    from diff_samples import render
    from raytracinginoneweekendinrust_amd import _capi
    import exec_join_check
    from kernel_resources import readable
    fixture = os.path.join(LIB, "librtamd_rngdiv.so")
    assert os.path.exists(fixture), "make -C raytracinginoneweekendinrust_amd/csrc rngdiv"
    # the fixture reproduces the miscompile only where this compiler splits the join that way
    # (tests/test_exec_join.py reports it); render the preset whose instance is split, or skip
    split = {readable(fn) for fn, _, _ in exec_join_check.check_library(fixture)}
    if split & {"trace_samples<0, 3, 63>", "trace_samples<0, 4, 63>"}:
        _all_features_fixture(rt, orc, bind(_capi.LIB_PATH, 0), bind(fixture, 1), _capi)
        return
    if not split:  # the compiler no longer splits that join (tests/test_exec_join.py reports it)
        pytest.skip("the live fixture has no split join on this compiler")
    # a preset's instance: that config at a reduced width, the fixture forced onto the split
    # instance's wave count (RT_OPT_TUNE kModeW3 = 0x40 / kModeW4 = 0x400000)
    presets = preset_configs()
    for inst in sorted(split):
        if not inst.startswith("trace_samples<0, "):
            continue
        waves, kf = inst[len("trace_samples<0, "):-1].split(", ")
        if int(kf.rstrip("u")) in presets:
            tune = "0x40" if waves == "3" else "0x400000"
            _config_fixture(rt, orc, presets[int(kf.rstrip("u"))], bind(_capi.LIB_PATH, 0),
                            bind(f"{fixture}:{tune}", 1), render)
            return
    raise AssertionError(f"the live fixture splits instances this test cannot render: {sorted(split)}")


def preset_configs():
    """kF preset value -> the BASELINE config that runs that fast-kernel instance, with the values
    taken from kernel.hip's kF constants (fast_instance), so a changed bit fails here instead of
    silently skipping."""
    import re
    src = open(os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "csrc", "kernel.hip")).read()
    kf = {m.group(1): int(m.group(2)) for m in re.finditer(r"\b(kF[A-Za-z]+) = (\d+)u\b", src)}
    for name in ("kFBvh", "kFTri", "kFRuns", "kFDeep", "kFMarble", "kFSusp"):
        assert name in kf, name
    return {kf["kFBvh"]: "C1", kf["kFBvh"] | kf["kFMarble"]: "C3",
            kf["kFBvh"] | kf["kFTri"] | kf["kFDeep"] | kf["kFSusp"]: "C4", 0: "C5", kf["kFRuns"]: "C2"}


def _all_features_fixture(rt, orc, prod, fix, _capi):
    """The same check on the all-features instance: test_gpu_parity's every-preset scene (a long
    sphere run, a BVH and a triangle), rendered through each library's own C ABI."""
    import ctypes as C
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
    w.add(b.tri((-6, -1, -3), (6, -1, -3), (0, 4, -3), white))
    w.add(b.sphere((0, -1000.5, 0), 1000.0, white))
    sc = b.finish(w)
    cam = rt.Camera.new((0, 2, 9), (0, 0.5, 0), (0, 1, 0), 45.0, 1.5, 0.05, 9.0, 0.0, 0.0)

    def render(lib, depth):
        h = C.c_void_p()
        assert lib.rt_scene_upload(sc.desc, 0, C.byref(h)) == 0
        p = rt.render_params(96, 64, 8, depth, background=(0.6, 0.7, 0.9))
        img = np.zeros(96 * 64 * 3, dtype=np.float32)
        st = _capi.rt_stats()
        d = cam.desc()
        assert lib.rt_render(h, C.byref(d), C.byref(p), img.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)) == 0
        lib.rt_scene_free(h)
        return img

    def oracle(depth):
        return np.asarray(orc.render(sc, cam, rt.render_params(96, 64, 8, depth, background=(0.6, 0.7, 0.9)))[0]).ravel()

    want = oracle(12)
    np.testing.assert_array_equal(render(prod, 12), want)
    got = render(fix, 12)
    same = (got == want) | (np.isnan(got) & np.isnan(want))
    assert not same.all(), "the split copies left every lane's Rng buffer intact"


def _config_fixture(rt, orc, name, prod, fix, render):
    """One sample index of config `name` at width 240: the product renders the oracle's image and
    the fixture does not. (Where the split join sits decides which segment goes wrong first: in
    C1's instance it came after the camera segment, in C3's 3-wave instance the camera segment
    itself already differs in 78 of 115,200 values; so no case checks a particular depth.)"""
    cfg = rt.CONFIGS[name]
    cfg = cfg.scaled(240, 1)
    from raytracinginoneweekendinrust_amd import _capi
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)

    def oracle(depth):
        p = rt.render_params(cfg.width, cfg.height, 1, depth, background=cfg.background(), seed=cfg.render_seed,
                             sample_base=0)
        img, _ = orc.render(scene, cfg.camera(), p, threads=8)
        return img.reshape(cfg.height, cfg.width, 3)

    want = oracle(cfg.depth)
    np.testing.assert_array_equal(render(prod, cfg, rt, _capi, 0)[0], want)
    got = render(fix, cfg, rt, _capi, 0)[0]
    same = (got == want) | (np.isnan(got) & np.isnan(want))
    assert not same.all(), "the split copies left every lane's Rng buffer intact"
