"""Diagnostic options for the tools (not the product): the library reads no environment
variables (include/rt.h rt_set_option), so the session scripts' RT_TUNE=..., RT_GROUP=...,
RT_STACK_LDS=..., RT_SAMPLE_BUFFER_MB=..., RT_HRPP_SLOT_BITS=..., RT_LAUNCH_LOG=1 and
RT_BVH_BUILD=host|device|auto are turned into rt_set_option calls here, by the tool."""
import os

ENV = {"RT_TUNE": "tune", "RT_GROUP": "group", "RT_STACK_LDS": "stack_lds", "RT_SAMPLE_BUFFER_MB": "sample_buffer_mb",
       "RT_HRPP_SLOT_BITS": "hrpp_slot_bits", "RT_LAUNCH_LOG": "launch_log", "RT_BVH_BUILD": "bvh_build",
       "RT_GUIDE": "guide", "RT_BVH_SHAPE": "bvh_shape"}
OPT_IDS = {"tune": 0, "group": 1, "stack_lds": 2, "sample_buffer_mb": 3, "hrpp_slot_bits": 4, "launch_log": 5,
           "bvh_build": 6, "guide": 7, "bvh_shape": 8}


def from_env() -> dict:
    out = {}
    for var, name in ENV.items():
        v = os.environ.get(var)
        if v is None:
            continue
        out[name] = {"auto": 0, "host": 1, "device": 2}[v] if name == "bvh_build" else int(v, 0)
    return out


def apply(rt) -> dict:
    """Set the options named in the environment through the package (rt.set_option)."""
    opts = from_env()
    for k, v in opts.items():
        rt.set_option(k, v)
    return opts


def apply_lib(lib) -> None:
    """The same through a raw ctypes handle of a librtamd build (tools/ab_time.py); builds
    older than rt_set_option are left at their defaults."""
    import ctypes as C
    if not hasattr(lib, "rt_set_option"):
        return
    lib.rt_set_option.argtypes = [C.c_int, C.c_int64]
    for k, v in from_env().items():
        lib.rt_set_option(OPT_IDS[k], v)
