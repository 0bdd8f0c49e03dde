"""ctypes mirror of include/rt.h (the C ABI of the MI355X hot path).

Loads the in-tree ``_lib/librtamd.so`` built by ``csrc/Makefile``. There is no
Python or CPU fallback: if the library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "_lib")
# RT_LIBRARY selects a diagnostic build of the same ABI (e.g. _lib/librtamd_prof.so, tools/region_profile.py).
LIB_PATH = os.environ.get("RT_LIBRARY") or os.path.join(LIB_DIR, "librtamd.so")
ASSET_DIR = os.path.normpath(os.path.join(_HERE, "..", "assets"))

# rt_node_kind
RT_TEX_SOLID, RT_TEX_CHECKER, RT_TEX_MARBLE, RT_TEX_IMAGE = 1, 2, 3, 4
RT_MAT_LAMBERTIAN, RT_MAT_METAL, RT_MAT_DIELECTRIC, RT_MAT_DIFFUSE_LIGHT, RT_MAT_ISOTROPIC = 16, 17, 18, 19, 20
(RT_OBJ_SPHERE, RT_OBJ_MOVING_SPHERE, RT_OBJ_XY_RECT, RT_OBJ_XZ_RECT, RT_OBJ_YZ_RECT, RT_OBJ_CUBE, RT_OBJ_TRI,
 RT_OBJ_LIST, RT_OBJ_BVH, RT_OBJ_TRANSLATE, RT_OBJ_ROTATE_Y, RT_OBJ_CONSTANT_MEDIUM, RT_OBJ_BVH_TREE) = range(32, 45)
RT_BVH_LEFT_HITTABLE, RT_BVH_RIGHT_HITTABLE = 1, 2
ABI_VERSION = 2

RT_FLAG_EXACT_BVH = 1
RT_FLAG_HRPP = 2
RT_FLAG_ACCUMULATE = 4
RT_FLAG_RAW_SUM = 8
RT_FLAG_FRAMES_IN_FLIGHT = 16

# rt_option (rt_set_option): the library's diagnostic switches; it reads no environment
OPTIONS = {"tune": 0, "group": 1, "stack_lds": 2, "sample_buffer_mb": 3, "hrpp_slot_bits": 4, "launch_log": 5,
           "bvh_build": 6, "guide": 7, "bvh_shape": 8}

STATUS = {0: "RT_OK", -1: "RT_ERR_INVALID", -2: "RT_ERR_UNSUPPORTED", -3: "RT_ERR_HIP", -4: "RT_ERR_OOM",
          -5: "RT_ERR_NO_DEVICE", -6: "RT_ERR_IO"}


class rt_node(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("ref", C.c_int32 * 3), ("f", C.c_float * 12), ("seed", C.c_uint64)]


class rt_bvh_node(C.Structure):
    _fields_ = [("left", C.c_int32), ("right", C.c_int32), ("flags", C.c_uint32), ("parent", C.c_int32),
                ("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3)]


class rt_scene_desc(C.Structure):
    _fields_ = [("nodes", C.POINTER(rt_node)), ("num_nodes", C.c_uint32), ("world", C.c_int32),
                ("list_items", C.POINTER(C.c_int32)), ("num_list_items", C.c_uint32), ("reserved0", C.c_uint32),
                ("image_data", C.POINTER(C.c_uint8)), ("image_bytes", C.c_uint64),
                ("bvh_nodes", C.POINTER(rt_bvh_node)), ("num_bvh_nodes", C.c_uint32), ("reserved1", C.c_uint32)]


class rt_camera_desc(C.Structure):
    _fields_ = [("look_from", C.c_float * 3), ("look_at", C.c_float * 3), ("view_up", C.c_float * 3),
                ("vfov_deg", C.c_float), ("aspect_ratio", C.c_float), ("aperture", C.c_float),
                ("focus_dist", C.c_float), ("time0", C.c_float), ("time1", C.c_float)]


class rt_camera(C.Structure):
    """The nine fields of the reference's Camera (src/camera.rs:6-27)."""
    _fields_ = [("origin", C.c_float * 3), ("horizontal", C.c_float * 3), ("vertical", C.c_float * 3),
                ("lower_left_corner", C.c_float * 3), ("u", C.c_float * 3), ("v", C.c_float * 3),
                ("lens_radius", C.c_float), ("time_start", C.c_float), ("time_end", C.c_float)]


class rt_render_params(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("samples_per_pixel", C.c_uint32),
                ("max_depth", C.c_uint32), ("tile_width", C.c_uint32), ("tile_height", C.c_uint32),
                ("seed", C.c_uint64), ("sample_base", C.c_uint32), ("shard_index", C.c_uint32),
                ("shard_count", C.c_uint32), ("flags", C.c_uint32), ("background", C.c_float * 3),
                ("spp_total", C.c_uint32)]


class rt_stats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("samples", C.c_uint64), ("kernel_ms", C.c_double)]


class rt_tile(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("x_start", C.c_uint32), ("y_start", C.c_uint32)]


assert C.sizeof(rt_node) == 72
assert C.sizeof(rt_render_params) == 64
assert C.sizeof(rt_bvh_node) == 40
assert C.sizeof(rt_scene_desc) == 64
assert C.sizeof(rt_camera) == 84

# (name, restype, argtypes) for every symbol declared in include/rt.h
SIGNATURES = [
    ("rt_abi_version", C.c_int, []),
    ("rt_last_error", C.c_char_p, []),
    ("rt_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("rt_tile_image", C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(rt_tile), C.c_uint32,
                                C.POINTER(C.c_uint32)]),
    ("rt_scene_upload", C.c_int, [C.POINTER(rt_scene_desc), C.c_int, C.POINTER(C.c_void_p)]),
    ("rt_scene_free", C.c_int, [C.c_void_p]),
    ("rt_scene_info", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    ("rt_render_launch", C.c_int, [C.c_void_p, C.POINTER(rt_camera_desc), C.POINTER(rt_render_params), C.c_void_p,
                                   C.c_void_p, C.c_void_p]),
    ("rt_render_multi", C.c_int, [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(rt_camera_desc),
                                  C.POINTER(rt_render_params), C.POINTER(C.c_float), C.POINTER(rt_stats)]),
    ("rt_quantize_srgb8", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]),
    ("rt_format_ppm", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64),
                                C.c_void_p]),
    ("rt_scene_trace_time", C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_int]),
    ("rt_render", C.c_int, [C.c_void_p, C.POINTER(rt_camera_desc), C.POINTER(rt_render_params),
                            C.POINTER(C.c_float), C.POINTER(rt_stats)]),
    ("rt_scene_generate", C.c_int, [C.c_char_p, C.c_uint64, C.c_char_p, C.POINTER(C.POINTER(rt_scene_desc))]),
    ("rt_scene_desc_free", None, [C.POINTER(rt_scene_desc)]),
    ("rt_scene_background", C.c_int, [C.c_char_p, C.POINTER(C.c_float)]),
    ("rt_scene_hrpp_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint32)]),
    ("rt_bvh_build_order", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p, C.c_void_p]),
    ("rt_device_numeric_eval", C.c_int, [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                         C.POINTER(C.c_double), C.c_uint32]),
    ("rt_camera_new", C.c_int, [C.POINTER(rt_camera_desc), C.POINTER(rt_camera)]),
    ("rt_render_camera", C.c_int, [C.c_void_p, C.POINTER(rt_camera), C.POINTER(rt_render_params),
                                   C.POINTER(C.c_float), C.POINTER(rt_stats)]),
    ("rt_render_launch_camera", C.c_int, [C.c_void_p, C.POINTER(rt_camera), C.POINTER(rt_render_params), C.c_void_p,
                                          C.c_void_p, C.c_void_p]),
    ("rt_render_multi_camera", C.c_int, [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(rt_camera),
                                         C.POINTER(rt_render_params), C.POINTER(C.c_float), C.POINTER(rt_stats)]),
    ("rt_shard_floats", C.c_uint64, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("rt_shard_offset", C.c_uint64, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("rt_shard_pack", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("rt_shard_unpack", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("rt_ipc_export", C.c_int, [C.c_void_p, C.c_int, C.c_char_p]),
    ("rt_ipc_open", C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]),
    ("rt_ipc_close", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_copy_async", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    ("rt_shard_pull_unpack", C.c_int, [C.POINTER(C.c_void_p), C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                       C.c_void_p]),
    ("rt_device_kat", C.c_int, [C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_uint32]),
    ("rt_set_option", C.c_int, [C.c_int, C.c_int64]),
    ("rt_get_option", C.c_int, [C.c_int, C.POINTER(C.c_int64)]),
]


def load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the MI355X path has no CPU fallback)")
    # One HIP runtime per process. torch ships its own libamdhip64 (soname libamdhip64.so.7,
    # file name libamdhip64.so); loading torch first lets librtamd's NEEDED entry bind to that
    # copy by soname. Loaded the other way round, the process holds two runtimes and whichever
    # initialises second finds no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rt_abi_version() != ABI_VERSION:
        raise ImportError("librtamd.so ABI version mismatch")
    return lib


lib = load()


class RTError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = lib.rt_last_error().decode(errors="replace")
        super().__init__(f"{where}: {STATUS.get(code, code)}: {msg}")
        self.code = code


def check(code: int, where: str) -> None:
    if code != 0:
        raise RTError(code, where)
