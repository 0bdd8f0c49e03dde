#!/usr/bin/env python3
"""Diagnostic: a C3 frame (reduced spp) rendered with the default block order (last block
first) and with RT_OPT_TUNE bit 21 (top-first, the earlier order) must be the same bits."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import raytracinginoneweekendinrust_amd as rt
    cfg = rt.CONFIGS["C3"].scaled(rt.CONFIGS["C3"].width, 16)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    imgs = []
    for tune in (0, 1 << 21):
        rt.set_option("tune", tune)
        ds = rt.DeviceScene(scene)
        p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                             seed=cfg.render_seed)
        imgs.append(ds.render(cfg.camera(), p)[0])
        ds.close()
    rt.set_option("tune", 0)
    a, b = (np.asarray(i).view(np.uint32) for i in imgs)
    print("block orders: identical bits" if np.array_equal(a, b) else
          f"block orders: {int((a != b).sum())} words differ", flush=True)


if __name__ == "__main__":
    main()
