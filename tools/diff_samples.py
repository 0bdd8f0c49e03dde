#!/usr/bin/env python3
"""Locate the samples and the bounce where two librtamd builds disagree (diagnostic, GPU box).

    python3 tools/diff_samples.py --config C1 [--samples 50] [--depth-sweep 8] good.so bad.so

Renders the config one sample index at a time (spp 1, sample_base s: every pixel's sample s,
the same Philox stream as in the full frame) with both libraries and lists the (pixel, sample)
pairs whose radiance differs, with the CPU oracle's value for each, so the build that left the
reference's result is named. For the first differing pair it then renders that sample with
max_depth 1, 2, ... and reports the first depth at which the two builds differ: the bounce
whose list walk, traversal or scatter computed something else.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")]
from ab_time import bind  # noqa: E402


def render(lib, cfg, rt, _capi, sample, depth=None):
    desc = C.POINTER(_capi.rt_scene_desc)()
    assert lib.rt_scene_generate(cfg.scene.encode(), cfg.scene_seed, _capi.ASSET_DIR.encode(), C.byref(desc)) == 0
    h = C.c_void_p()
    assert lib.rt_scene_upload(desc, 0, C.byref(h)) == 0
    p = rt.render_params(cfg.width, cfg.height, 1, depth or cfg.depth, background=cfg.background(),
                         seed=cfg.render_seed, sample_base=sample)
    img = np.zeros(cfg.width * cfg.height * 3, dtype=np.float32)
    st = _capi.rt_stats()
    cam = cfg.camera().desc()
    assert lib.rt_render(h, C.byref(cam), C.byref(p), img.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)) == 0
    lib.rt_scene_free(h)
    return img.reshape(cfg.height, cfg.width, 3), st.segments


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1")
    ap.add_argument("--samples", type=int, default=50)
    ap.add_argument("--depth-sweep", type=int, default=12)
    ap.add_argument("libs", nargs=2)
    a = ap.parse_args()
    import oracle_ffi as orc
    import raytracinginoneweekendinrust_amd as rt
    from raytracinginoneweekendinrust_amd import _capi
    cfg = rt.CONFIGS[a.config]
    libs = [bind(p, i) for i, p in enumerate(a.libs)]
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    first = None
    total = 0
    for s in range(a.samples):
        (ia, sa), (ib, sb) = (render(lib, cfg, rt, _capi, s) for lib in libs)
        bad = np.argwhere((ia != ib).any(axis=2) & ~(np.isnan(ia) & np.isnan(ib)).all(axis=2))
        total += len(bad)
        if len(bad):
            p = rt.render_params(cfg.width, cfg.height, 1, cfg.depth, background=cfg.background(),
                                 seed=cfg.render_seed, sample_base=s)
            want, _ = orc.render(scene, cfg.camera(), p, threads=8)
            want = want.reshape(cfg.height, cfg.width, 3)
            y, x = bad[0]
            print(f"sample {s}: {len(bad)} pixels differ, segments {sa} vs {sb}; first (x={x}, y={y}): "
                  f"A {ia[y, x].tolist()} B {ib[y, x].tolist()} oracle {want[y, x].tolist()}; "
                  f"A==oracle on {int((ia[bad[:, 0], bad[:, 1]] == want[bad[:, 0], bad[:, 1]]).all(axis=1).sum())}, "
                  f"B==oracle on {int((ib[bad[:, 0], bad[:, 1]] == want[bad[:, 0], bad[:, 1]]).all(axis=1).sum())} "
                  f"of them", flush=True)
            if first is None:
                first = (s, int(x), int(y))
    print(f"total differing (pixel, sample) pairs: {total}", flush=True)
    if first is None:
        return
    s, x, y = first
    for d in range(1, a.depth_sweep + 1):
        (ia, _), (ib, _) = (render(lib, cfg, rt, _capi, s, depth=d) for lib in libs)
        print(f"sample {s} pixel ({x}, {y}) depth {d}: A {ia[y, x].tolist()} B {ib[y, x].tolist()}"
              f"{'  <- first difference' if (ia[y, x] != ib[y, x]).any() else ''}", flush=True)
        if (ia[y, x] != ib[y, x]).any():
            break


if __name__ == "__main__":
    main()
