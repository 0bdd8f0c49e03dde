"""The output step and the single-process multi-device render, on a real MI355X.

rt_format_ppm / rt_quantize_srgb8 (src/renderer.rs:107-127, palette 0.6.1 f32 -> u8)
against the oracle's restatement (oracle_ffi.srgb8 / ppm), byte for byte; and
rt_render_multi against the one-device render, bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle_ffi

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def edge_image():
    """Every f32 region the conversion distinguishes: NaN, +-inf, +-0, negatives,
    denormals, the rounding boundary of each code, exactly 1, just above 1, huge."""
    vals = [np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, -1e-30, -0.5, 1e-45, 1e-38, 1.0, 1.0000001, 2.0, 3e38]
    k = np.arange(256, dtype=np.float32)
    for d in (-1e-7, 0.0, 1e-7):                      # (k + 0.5) / 255 +- a little: the half-way ties
        vals += list(((k + np.float32(0.5)) / np.float32(255.0)) + np.float32(d))
    vals += list(k / np.float32(255.0))
    v = np.array(vals, dtype=np.float32)
    v = np.concatenate([v, np.zeros((-len(v)) % 3, np.float32)])
    return v.reshape(1, -1, 3)


def test_quantize_matches_palette_on_edge_values(rt):
    img = edge_image()
    np.testing.assert_array_equal(rt.quantize_srgb8(img), oracle_ffi.srgb8(img))


def test_format_ppm_matches_write_ppm_on_edge_values(rt):
    img = edge_image()
    assert rt.format_ppm(img) == oracle_ffi.ppm(img)
    tall = np.ascontiguousarray(img.reshape(-1, 1, 3))  # one pixel per row: checks the row order
    assert rt.format_ppm(tall) == oracle_ffi.ppm(tall)


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (130, 67)])
def test_format_ppm_random_and_ragged(w, h, rt):
    rng = np.random.default_rng(w * 1000 + h)
    img = rng.uniform(-0.2, 1.2, size=(h, w, 3)).astype(np.float32)
    assert rt.format_ppm(img) == oracle_ffi.ppm(img)


def c3(rt, width, spp, scene_seed=None):
    cfg = rt.CONFIGS["C3"].scaled(width, spp)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed if scene_seed is None else scene_seed)
    params = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(), seed=3)
    return cfg, scene, params


def test_format_ppm_of_a_render(rt):
    cfg, scene, params = c3(rt, 96, 4)
    ds = rt.DeviceScene(scene)
    img, _ = ds.render(cfg.camera(), params)
    ds.close()
    assert rt.format_ppm(img) == oracle_ffi.ppm(img)


def test_format_ppm_full_frame(rt):
    # 1200 x 800 lines: the scan of line lengths spans many rocPRIM blocks
    rng = np.random.default_rng(7)
    img = rng.uniform(-0.05, 1.05, size=(800, 1200, 3)).astype(np.float32)
    assert rt.format_ppm(img) == oracle_ffi.ppm(img)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_render_multi_equals_one_device_render(n, rt):
    cfg, scene, params = c3(rt, 72, 3)
    one = rt.DeviceScene(scene)
    want, st1 = one.render(cfg.camera(), params)
    one.close()
    handles = [rt.DeviceScene(scene, 0) for _ in range(n)]  # n "devices", all device 0 on a 1-GPU box
    got, stn = rt.render_multi(handles, cfg.camera(), params)
    for h in handles:
        h.close()
    np.testing.assert_array_equal(got, want)
    assert stn["segments"] == st1["segments"]


def test_shimmer_cli_writes_the_reference_ppm(rt, tmp_path):
    # the CLI (main.rs flags) renders C3's camera at 64 px / 2 spp; its stdout must be
    # write_ppm of the library's render of the same scene, camera and seeds
    cfg, scene, params = c3(rt, 64, 2, scene_seed=3)  # --seed seeds both the scene and the samples
    exe = os.path.join(REPO, "raytracinginoneweekendinrust_amd", "_lib", "shimmer")
    pfm = tmp_path / "img.pfm"
    f3 = lambda v: [repr(float(x)) for x in v]
    args = [exe, cfg.scene, "-w", str(cfg.width), "-a", "3", "2", "-s", str(cfg.spp), "-d", str(cfg.depth),
            "--cam-look-from", *f3(cfg.look_from), "--cam-look-at", *f3(cfg.look_at), "--cam-vertical-fov",
            str(cfg.vfov), "--cam-start-time", str(cfg.time0), "--cam-end-time", str(cfg.time1),
            "--seed", "3", "--pfm", str(pfm)]
    r = subprocess.run(args, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    raw = pfm.read_bytes()
    head_end = raw.index(b"-1.0\n") + 5
    w, h = map(int, raw[3:head_end].split(b"\n")[0].split())
    img = np.frombuffer(raw[head_end:], dtype=np.float32).reshape(h, w, 3)
    assert r.stdout == oracle_ffi.ppm(img)
    ds = rt.DeviceScene(scene)
    want, _ = ds.render(cfg.camera(), params)
    ds.close()
    np.testing.assert_array_equal(img, want)


@pytest.mark.parametrize("slices", [[16], [8, 8], [3, 5, 8], [1] * 16])
def test_progressive_slices_equal_the_one_shot_render(slices, rt):
    # RT_FLAG_ACCUMULATE / RT_FLAG_RAW_SUM keep every pixel's sum in sample order,
    # so the last slice's image is the one-shot frame bit for bit
    cfg, scene, params = c3(rt, 64, 16)
    ds = rt.DeviceScene(scene)
    want, _ = ds.render(cfg.camera(), params)
    done, img = 0, None
    for done, img in rt.render_progressive(ds, cfg.camera(), params, slices):
        assert np.isfinite(img).all()
    ds.close()
    assert done == 16
    np.testing.assert_array_equal(img, want)
