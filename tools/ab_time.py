#!/usr/bin/env python3
"""A/B timing of librtamd builds on the same GPU (diagnostic).

    python3 tools/ab_time.py [--config C3] [--spp N] [--reps R] lib1.so [lib2.so ...]

Binds only the entry points every ABI-1 build exports (rt_scene_generate,
rt_scene_upload, rt_render) so older builds can be compared with the current
one on the same box; prints the median rt_render kernel time and checks that
every library produced the same image bits as the first.
"""
import argparse
import ctypes as C
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RT_LIBRARY", os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "_lib", "librtamd.so"))
from raytracinginoneweekendinrust_amd import _capi  # noqa: E402  (structs only)
from raytracinginoneweekendinrust_amd.configs import CONFIGS  # noqa: E402


def bind(spec, idx):
    """spec: path.so, or path.so:0xTUNE (that library's RT_OPT_TUNE bits, e.g. 0x40 = the 3-wave
    instance), or path.so:name=value,... (rt_set_option by tools/rtopts.py names, e.g.
    migrate=0). Each spec loads its own copy of the file, so one build can be compared with itself."""
    import shutil
    import tempfile
    path, _, tune = spec.partition(":")
    copy = os.path.join(tempfile.gettempdir(), f"ab_{os.getpid()}_{idx}_{os.path.basename(path)}")
    shutil.copyfile(path, copy)
    lib = C.CDLL(copy)
    os.unlink(copy)  # the mapping stays valid; nothing is left in the temp directory
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import rtopts
    rtopts.apply_lib(lib)
    if tune:
        lib.rt_set_option.argtypes = [C.c_int, C.c_int64]
        for item in tune.split(","):
            name, _, val = item.rpartition("=")
            rc = lib.rt_set_option(rtopts.OPT_IDS[name] if name else 0, int(val, 0))
            assert rc == 0, (spec, item, rc)
    lib.rt_scene_generate.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p, C.POINTER(C.POINTER(_capi.rt_scene_desc))]
    lib.rt_scene_upload.argtypes = [C.POINTER(_capi.rt_scene_desc), C.c_int, C.POINTER(C.c_void_p)]
    lib.rt_render.argtypes = [C.c_void_p, C.POINTER(_capi.rt_camera_desc), C.POINTER(_capi.rt_render_params),
                              C.POINTER(C.c_float), C.POINTER(_capi.rt_stats)]
    lib.rt_scene_free.argtypes = [C.c_void_p]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    import raytracinginoneweekendinrust_amd as rt
    cfg = CONFIGS[a.config]
    if a.spp:
        cfg = cfg.scaled(cfg.width, a.spp)
    cam = cfg.camera().desc()
    params = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                              seed=cfg.render_seed)
    ref = None
    for i, path in enumerate(a.libs):
        lib = bind(path, i)
        desc = C.POINTER(_capi.rt_scene_desc)()
        assert lib.rt_scene_generate(cfg.scene.encode(), cfg.scene_seed, _capi.ASSET_DIR.encode(), C.byref(desc)) == 0
        h = C.c_void_p()
        assert lib.rt_scene_upload(desc, 0, C.byref(h)) == 0
        img = np.zeros(cfg.width * cfg.height * 3, dtype=np.float32)
        times, segs = [], 0
        for _ in range(a.reps + 1):
            st = _capi.rt_stats()
            rc = lib.rt_render(h, C.byref(cam), C.byref(params), img.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st))
            assert rc == 0, rc
            times.append(st.kernel_ms)
            segs = st.segments
        med = statistics.median(times[1:])
        same = "first" if ref is None else ("identical" if np.array_equal(ref, img) else "DIFFERENT")
        if ref is None:
            ref = img.copy()
        samples = cfg.width * cfg.height * cfg.spp
        print(f"{os.path.basename(path):40s} {med:9.1f} ms  {samples / med / 1e3:8.1f} Msamples/s  "
              f"segments {segs}  image {same}", flush=True)
        lib.rt_scene_free(h)


if __name__ == "__main__":
    main()
