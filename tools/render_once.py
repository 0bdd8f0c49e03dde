#!/usr/bin/env python3
"""Render one BASELINE config on device 0 through the C ABI (profiling driver).

    python tools/render_once.py --config C3 [--spp 100] [--reps 1] [--exact-bvh]

Prints the kernel time (HIP events inside rt_render) and segment count to stderr.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--exact-bvh", action="store_true")
    a = ap.parse_args()
    import raytracinginoneweekendinrust_amd as rt
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import rtopts
    rtopts.apply(rt)  # RT_TUNE=... etc. of the session scripts -> rt_set_option
    cfg = rt.CONFIGS[a.config]
    cfg = cfg.scaled(a.width or cfg.width, a.spp or cfg.spp)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    ds = rt.DeviceScene(scene)
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                         exact_bvh=a.exact_bvh)
    for i in range(a.reps):
        img, st = ds.render(cfg.camera(), p)
        print(f"{cfg.name} {cfg.width}x{cfg.height}x{cfg.spp}: kernel {st['kernel_ms']:.2f} ms, "
              f"{st['samples'] / st['kernel_ms'] / 1e3:.1f} Msamples/s, {st['segments']} segments, "
              f"mean {img.mean():.5f}", file=sys.stderr)
    ds.close()


if __name__ == "__main__":
    main()
