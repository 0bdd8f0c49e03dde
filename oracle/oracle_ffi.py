"""ctypes loader for the CPU parity oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / reported CPU baseline. The
product package never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from raytracinginoneweekendinrust_amd import _capi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

FLAG_RECURSIVE = 1
FLAG_LIBM = 2


class oracle_options(C.Structure):
    _fields_ = [("flags", C.c_uint32), ("num_threads", C.c_uint32)]


class oracle_counters(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64), ("hits", C.c_uint64),
                ("node_visits", C.c_uint64), ("sphere_tests", C.c_uint64), ("msphere_tests", C.c_uint64),
                ("rect_tests", C.c_uint64), ("tri_tests", C.c_uint64), ("medium_tests", C.c_uint64),
                ("texel_fetches", C.c_uint64), ("seconds", C.c_double), ("threads", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load() -> C.CDLL:
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    P = C.POINTER
    lib.oracle_render.restype = C.c_int
    lib.oracle_render.argtypes = [P(_capi.rt_scene_desc), P(_capi.rt_camera_desc), P(_capi.rt_render_params),
                                  P(oracle_options), P(C.c_float), P(oracle_counters)]
    lib.oracle_render_camera.restype = C.c_int
    lib.oracle_render_camera.argtypes = [P(_capi.rt_scene_desc), P(_capi.rt_camera), P(_capi.rt_render_params),
                                         P(oracle_options), P(C.c_float), P(oracle_counters)]
    lib.oracle_sample.restype = C.c_int
    lib.oracle_sample.argtypes = [P(_capi.rt_scene_desc), P(_capi.rt_camera_desc), P(_capi.rt_render_params),
                                  C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_float)]
    lib.oracle_last_error.restype = C.c_char_p
    lib.oracle_philox4x32_10.argtypes = [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
    lib.oracle_philox4x32_10.restype = None
    lib.oracle_tile.restype = C.c_uint32
    lib.oracle_tile.argtypes = [C.c_uint32] * 4 + [P(_capi.rt_tile), C.c_uint32]
    lib.oracle_aabb_hit.restype = C.c_int
    lib.oracle_aabb_hit.argtypes = [P(C.c_float)] * 4 + [C.c_float, C.c_float]
    lib.oracle_aabb_union.restype = C.c_int
    lib.oracle_aabb_union.argtypes = [P(C.c_float), P(C.c_float), P(C.c_float)]
    lib.oracle_sphere_uv.restype = None
    lib.oracle_sphere_uv.argtypes = [P(C.c_float), P(C.c_float)]
    lib.oracle_camera_basis.restype = None
    lib.oracle_camera_basis.argtypes = [P(_capi.rt_camera_desc), P(C.c_float)]
    lib.oracle_turbulence.restype = C.c_double
    lib.oracle_turbulence.argtypes = [C.c_uint32, P(C.c_double)]
    return lib


lib = _load()


def _check(rc: int, where: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{where}: {rc}: {lib.oracle_last_error().decode(errors='replace')}")


def render(scene, camera, params, *, flags: int = 0, threads: int = 0, out: np.ndarray | None = None):
    """Oracle render of the shard selected by params; returns (image (H,W,3) f32, counters dict)."""
    if out is None:
        out = np.zeros((params.height, params.width, 3), dtype=np.float32)
    opt = oracle_options(flags, threads)
    cnt = oracle_counters()
    if hasattr(camera, "fields"):  # a constructed Camera (CameraBasis)
        cam = camera.fields()
        _check(lib.oracle_render_camera(scene.desc, C.byref(cam), C.byref(params), C.byref(opt),
                                        out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(cnt)), "oracle_render_camera")
    else:
        cam = camera.desc()
        _check(lib.oracle_render(scene.desc, C.byref(cam), C.byref(params), C.byref(opt),
                                 out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(cnt)), "oracle_render")
    return out, cnt.as_dict()


def sample(scene, camera, params, x: int, y: int, s: int, *, flags: int = 0) -> np.ndarray:
    rgb = (C.c_float * 3)()
    cam = camera.desc()
    _check(lib.oracle_sample(scene.desc, C.byref(cam), C.byref(params), flags, x, y, s, rgb), "oracle_sample")
    return np.array(rgb[:], dtype=np.float32)


def philox(ctr, key) -> list:
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib.oracle_philox4x32_10(c, k, o)
    return list(o)


def tile(w, h, tw, th):
    n = lib.oracle_tile(w, h, tw, th, None, 0)
    arr = (_capi.rt_tile * max(n, 1))()
    lib.oracle_tile(w, h, tw, th, arr, n)
    return [(t.width, t.height, t.x_start, t.y_start) for t in arr[:n]]


def aabb_hit(mn, mx, o, d, tmin, tmax) -> bool:
    f = lambda v: (C.c_float * 3)(*v)
    return bool(lib.oracle_aabb_hit(f(mn), f(mx), f(o), f(d), tmin, tmax))


def aabb_union(a, b):
    f = lambda v: None if v is None else (C.c_float * 6)(*v)
    out = (C.c_float * 6)()
    if not lib.oracle_aabb_union(f(a), f(b), out):
        return None
    return tuple(out)


def sphere_uv(p):
    uv = (C.c_float * 2)()
    lib.oracle_sphere_uv((C.c_float * 3)(*p), uv)
    return uv[0], uv[1]


def camera_basis(camera) -> np.ndarray:
    out = (C.c_float * 21)()
    cam = camera.desc()
    lib.oracle_camera_basis(C.byref(cam), out)
    return np.array(out[:], dtype=np.float32)


def turbulence(seed: int, p) -> float:
    return lib.oracle_turbulence(seed, (C.c_double * 3)(*p))


lib.oracle_numeric_eval.restype = None
lib.oracle_numeric_eval.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                    C.c_uint32]


def numeric_eval(op: int, a, b=None) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    bp = None
    if b is not None:
        b = np.ascontiguousarray(b, dtype=np.float64)
        bp = b.ctypes.data_as(C.POINTER(C.c_double))
    lib.oracle_numeric_eval(op, a.ctypes.data_as(C.POINTER(C.c_double)), bp,
                            out.ctypes.data_as(C.POINTER(C.c_double)), a.size)
    return out


def srgb8(img: np.ndarray) -> np.ndarray:
    """palette 0.6.1 `Srgb::<f32>::into_format::<u8>()` per channel, as called by
    Renderer::write_ppm (src/renderer.rs:116-121; srgb_from_vec3 applies no gamma,
    src/utils.rs:19-23): scaled = c * 255.0 in f32, f32::round (half away from zero),
    clamp to [0, 255], `as u8` (NaN -> 0). Rows are returned top to bottom (y = H-1
    first), the order write_ppm emits them. Restated in the reference's own order
    (scale, round, clamp), so it also checks the device's clamp-first evaluation."""
    with np.errstate(over="ignore", invalid="ignore"):   # 3e38 * 255 -> inf, as in f32 on the device
        s = np.asarray(img, dtype=np.float32)[::-1] * np.float32(255.0)
    a = np.abs(s).astype(np.float64)          # f32 -> f64 is exact; +0.5 then floor is exact too
    r = np.copysign(np.floor(a + 0.5), s)
    r = np.where(r < 0.0, 0.0, np.where(r > 255.0, 255.0, r))
    return np.nan_to_num(r, nan=0.0).astype(np.uint8)


def ppm(img: np.ndarray) -> bytes:
    """Renderer::write_ppm (src/renderer.rs:107-127): "P3\\nW H\\n255\\n" then "r g b\\n" per pixel."""
    h, w, _ = img.shape
    q = srgb8(img).reshape(-1, 3)
    body = "".join(f"{r} {g} {b}\n" for r, g, b in q.tolist())
    return f"P3\n{w} {h}\n255\n{body}".encode()


lib.oracle_bvh_order.restype = C.c_int
lib.oracle_bvh_order.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p]


def bvh_order(keys: np.ndarray, seed: int) -> np.ndarray:
    """Leaf order of Bvh::new (bvh.rs:249-333) for box_compare keys (n, 3) float32."""
    keys = np.ascontiguousarray(keys, dtype=np.float32).reshape(-1, 3)
    out = np.empty(len(keys), dtype=np.uint32)
    _check(lib.oracle_bvh_order(keys.ctypes.data, len(keys), seed, out.ctypes.data), "oracle_bvh_order")
    return out
