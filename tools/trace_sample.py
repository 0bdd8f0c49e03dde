#!/usr/bin/env python3
"""Render one sample index of a config with one librtamd build (diagnostic, GPU box).

    python3 tools/trace_sample.py --config C1 --sample 0 --x 3 --y 0 lib.so

Paired with a build compiled with -DRT_DEBUG_PIXEL=<y*width+x>u -DRT_DEBUG_SAMPLE=<s>u (the
device printf in finish_segment prints each segment's ray, hit flag, entry, leaf code and t as
float bits) and with oracle.c built with -DORACLE_TRACE (the same lines from ray_color_fwd),
so the first segment where a build leaves the reference's path is read off directly.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
from diff_samples import render  # noqa: E402
from ab_time import bind  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1")
    ap.add_argument("--sample", type=int, default=0)
    ap.add_argument("--x", type=int, default=3)
    ap.add_argument("--y", type=int, default=0)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("lib")
    a = ap.parse_args()
    import raytracinginoneweekendinrust_amd as rt
    from raytracinginoneweekendinrust_amd import _capi
    cfg = rt.CONFIGS[a.config]
    img, segs = render(bind(a.lib, 0), cfg, rt, _capi, a.sample, depth=a.depth)
    print(f"{os.path.basename(a.lib)} pixel ({a.x}, {a.y}) sample {a.sample}: {img[a.y, a.x].tolist()} "
          f"segments {segs}", flush=True)


if __name__ == "__main__":
    main()
