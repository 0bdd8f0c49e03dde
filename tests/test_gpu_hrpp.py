"""The HRPP experiment (RT_FLAG_HRPP: src/hrpp.rs, src/bvh.rs:114-211) on a real MI355X.

HRPP is approximate and its tables fill concurrently, so it has no bit-exact
oracle (nor does the reference: bvh.rs:146-149). What is pinned here:
* the ray hash's float mapping, bit for bit against a restatement of
  hrpp.rs:136-170 (BitPrecision::Six);
* with no table (rt_set_option(RT_OPT_HRPP_SLOT_BITS, 0)) every call is a "no prediction" and the
  render is bit-identical to the exact path — the predictor plumbing changes
  nothing by itself;
* scenes without Bvh::with_predictor are untouched by the flag;
* with tables, predictions happen, the statistics add up, and the image stays
  close to the exact one (tolerance below; measured error is reported by
  tools/hrpp_experiment.py).
"""
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def map_float_to_hash(v: float) -> int:
    """hrpp.rs:136-170 with BitPrecision::Six: shift 25 / 17, mask 0x3f."""
    bits = struct.unpack("<I", struct.pack("<f", v))[0]
    sign = (bits >> 31) & 1
    exp = (bits >> 25) & 0x3F
    man = (bits >> 17) & 0x3F
    return (sign << 15) | (exp << 7) | man


def test_hash_float_mapping_matches_hrpp_rs(rt):
    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.normal(size=2000) * 10 ** rng.uniform(-6, 6, 2000),
                           [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, 1e-45, 3.4e38, 0.5, 478.0, -600.0]])
    vals = vals.astype(np.float32).astype(np.float64)
    got = rt.numeric_eval(8, vals)
    want = np.array([map_float_to_hash(float(v)) for v in vals], dtype=np.float64)
    np.testing.assert_array_equal(got, want)


def c3(rt, width, spp):
    cfg = rt.CONFIGS["C3"].scaled(width, spp)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    return cfg, scene


def render(rt, scene, cfg, bits=None, **kw):
    with rt.options(**({} if bits is None else {"hrpp_slot_bits": bits})):
        ds = rt.DeviceScene(scene)
        p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(), **kw)
        img, st = ds.render(cfg.camera(), p)
        stats = ds.hrpp_stats()
        ds.close()
    return img, st, stats


def test_without_a_table_hrpp_equals_the_exact_path(rt):
    cfg, scene = c3(rt, 96, 8)
    exact, se, _ = render(rt, scene, cfg, exact_bvh=True)
    img, sh, stats = render(rt, scene, cfg, bits=0, hrpp=True)
    np.testing.assert_array_equal(img, exact)
    assert sh["segments"] == se["segments"]
    assert len(stats) == 2
    for s in stats:
        assert s["true_positive"] == 0 and s["false_positive"] == 0 and s["no_prediction"] > 0
        assert s["table_entries"] == 0 and s["predicted_nodes"] == 0


def test_scenes_without_predictors_ignore_the_flag(rt):
    cfg = rt.CONFIGS["C1"].scaled(64, 4)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    a, _, _ = render(rt, scene, cfg)
    b, _, stats = render(rt, scene, cfg, hrpp=True)
    np.testing.assert_array_equal(a, b)
    assert stats == []


def test_predictions_happen_and_the_image_stays_close(rt):
    cfg, scene = c3(rt, 120, 32)
    exact, _, _ = render(rt, scene, cfg, exact_bvh=True)
    img, _, stats = render(rt, scene, cfg, hrpp=True)
    assert np.isfinite(img).all()
    for s in stats:
        calls = s["true_positive"] + s["false_positive"] + s["no_prediction"]
        assert calls > 0 and s["true_positive"] > 0 and s["table_entries"] > 0
        assert s["table_entries"] <= s["predicted_nodes"] <= 6 * s["table_entries"]
    # tolerance: the mean over the frame of |HRPP - exact| on clamp01 colours stays
    # within 0.05 (noise at 32 spp is of that order; a wrong traversal is far larger)
    d = np.abs(np.clip(img, 0, 1) - np.clip(exact, 0, 1)).mean()
    assert d < 0.05, d
