"""The C-ABI library loads, exports exactly what include/rt.h declares, and reports
errors through rt_last_error without aborting (no device compute calls here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "rt.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(rt):
    from raytracinginoneweekendinrust_amd import _capi
    syms = declared_symbols()
    assert len(syms) == 35
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\sT\s(rt_[a-z0-9_]+)$", out.stdout, flags=re.M))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    assert {name for name, _, _ in _capi.SIGNATURES} == set(syms)


def test_library_is_built_for_gfx950(rt):
    from raytracinginoneweekendinrust_amd import _capi
    blob = open(_capi.LIB_PATH, "rb").read()
    # every embedded code object (offload bundle target id) is gfx950; rocPRIM's
    # host code carries arch-name string literals, so the check is on bundle ids only
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_abi_version(rt):
    assert rt.lib.rt_abi_version() == 2


def test_invalid_ir_is_reported_not_aborted(rt):
    b = rt.SceneBuilder()
    w = rt.HittableList()
    w.add(b.sphere((0, 0, 0), 1.0, 12345))  # material ref out of range
    sc = b.finish(w)
    with pytest.raises(rt.RTError) as e:
        rt.DeviceScene(sc)
    assert e.value.code == -1 and "range" in str(e.value)


def test_unsupported_bvh_leaf_is_reported(rt):
    b = rt.SceneBuilder()
    m = b.lambertian_from_color((0.5, 0.5, 0.5))
    inner = rt.HittableList()
    inner.add(b.sphere((0, 0, 0), 1.0, m))
    lst = rt.HittableList()
    lst.add(b.translate(b.sphere((0, 0, 0), 1.0, m), (1, 0, 0)))
    lst.add(b.sphere((3, 0, 0), 1.0, m))
    w = rt.HittableList()
    w.add(b.bvh(lst))
    with pytest.raises(rt.RTError) as e:
        rt.DeviceScene(b.finish(w))
    assert e.value.code == -2


def test_device_path_has_no_cpu_fallback(rt):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    sc = rt.Scene.generate("two-spheres", 1)
    with pytest.raises(rt.RTError) as e:
        rt.DeviceScene(sc)
    assert e.value.code == -5


def test_params_validation_happens_before_device_work(rt):
    from raytracinginoneweekendinrust_amd import _capi
    p = rt.render_params(0, 10, 1, 5)
    cam = rt.Camera().desc()
    out = np.zeros(30, dtype=np.float32)
    rc = rt.lib.rt_render(None, C.byref(cam), C.byref(p), out.ctypes.data_as(C.POINTER(C.c_float)), None)
    assert rc == -1
    assert rt.lib.rt_last_error()


def test_unknown_scene_and_background(rt):
    with pytest.raises(rt.RTError):
        rt.Scene.generate("no-such-scene", 1)
    with pytest.raises(rt.RTError):
        rt.scene_background("no-such-scene")
    assert rt.scene_background("showcase") == (0.0, 0.0, 0.0)
    assert rt.scene_background("random-spheres") == pytest.approx((0.7, 0.8, 1.0))


def test_missing_assets_is_io_error(rt, tmp_path):
    with pytest.raises(rt.RTError) as e:
        rt.Scene.generate("earth", 1, str(tmp_path))
    assert e.value.code == -6


def test_cli_usage_and_bad_flags():
    cli = os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "_lib", "shimmer")
    r = subprocess.run([cli, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--cam-look-from" in r.stderr
    r = subprocess.run([cli, "showcase", "--bogus"], capture_output=True, text=True)
    assert r.returncode == 2


def test_output_and_multi_entry_points_reject_bad_arguments(rt):
    # argument checks run before any HIP call, so these are safe without a GPU
    lib, INVALID = rt.lib, -1
    n = C.c_uint64(99)
    assert lib.rt_format_ppm(None, 4, 4, None, 0, C.byref(n), None) == INVALID
    dummy = C.c_void_p(1)
    assert lib.rt_format_ppm(dummy, 4, 4, dummy, 4 * 4 * 12 - 1, C.byref(n), None) == INVALID
    assert "12 bytes" in rt.lib.rt_last_error().decode()
    assert lib.rt_format_ppm(dummy, 0, 7, dummy, 0, C.byref(n), None) == 0 and n.value == 0
    assert lib.rt_quantize_srgb8(None, dummy, 1, 1, None) == INVALID
    cam = rt.CONFIGS["C3"].camera().desc()
    p = rt.render_params(8, 8, 1, 1)
    out = np.zeros(8 * 8 * 3, np.float32)
    assert lib.rt_render_multi(None, 1, C.byref(cam), C.byref(p), out.ctypes.data_as(C.POINTER(C.c_float)), None) == INVALID
    hs = (C.c_void_p * 2)(None, None)
    assert lib.rt_render_multi(hs, 0, C.byref(cam), C.byref(p), out.ctypes.data_as(C.POINTER(C.c_float)), None) == INVALID
    assert lib.rt_render_multi(hs, 2, C.byref(cam), C.byref(p), out.ctypes.data_as(C.POINTER(C.c_float)), None) == INVALID
    p2 = rt.render_params(8, 8, 1, 1, shard_index=0, shard_count=2)
    assert lib.rt_render_multi(hs, 2, C.byref(cam), C.byref(p2), out.ctypes.data_as(C.POINTER(C.c_float)), None) == INVALID
    assert "shards" in rt.lib.rt_last_error().decode()
    # the pull form of the gather: NULL arrays, more than 64 ranks and a NULL peer buffer of a
    # rank that owns blocks are refused before any launch; one rank has nothing to pull
    img = C.c_void_p(1)
    peers = (C.c_void_p * 65)(*([None] + [1] * 64))
    assert lib.rt_shard_pull_unpack(None, 16, 16, 2, img, None) == INVALID
    assert lib.rt_shard_pull_unpack(peers, 16, 16, 65, img, None) == INVALID
    assert "64 ranks" in rt.lib.rt_last_error().decode()
    holes = (C.c_void_p * 2)(None, None)
    assert lib.rt_shard_pull_unpack(holes, 16, 16, 2, img, None) == INVALID
    assert "peer buffer" in rt.lib.rt_last_error().decode()
    assert lib.rt_shard_pull_unpack(holes, 16, 16, 1, img, None) == 0


def test_one_hip_runtime_per_process(rt):
    # torch and librtamd must share one libamdhip64 (see _capi.load); two copies in one
    # process leave the second to initialise without a device
    import torch  # noqa: F401
    maps = open("/proc/self/maps").read()
    assert len(set(re.findall(r"\S*libamdhip64\S*", maps))) == 1


def test_diagnostic_options_are_explicit(rt):
    # rt_set_option replaces environment switches: the library's sources read no variable, an
    # unknown option or an out-of-range value is RT_ERR_INVALID, and options.__exit__
    # restores the previous values.
    from raytracinginoneweekendinrust_amd import _capi
    csrc = os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "csrc")
    for f in os.listdir(csrc):  # (rocPRIM's own host code may still consult its variables)
        if f.endswith((".hip", ".cpp", ".hpp")):
            assert "getenv" not in open(os.path.join(csrc, f)).read(), f
    assert rt.get_option("tune") == 0 and rt.get_option("hrpp_slot_bits") == -1
    with rt.options(guide=8):
        assert rt.get_option("guide") == 8
    assert rt.get_option("guide") == 0
    with rt.options(tune=1 << 16, stack_lds=2, bvh_build=1):
        assert (rt.get_option("tune"), rt.get_option("stack_lds"), rt.get_option("bvh_build")) == (1 << 16, 2, 1)
    assert (rt.get_option("tune"), rt.get_option("stack_lds"), rt.get_option("bvh_build")) == (0, 0, 0)
    for name, bad in (("group", 65), ("launch_log", 2), ("hrpp_slot_bits", 29), ("bvh_build", 3), ("stack_lds", -1),
                      ("guide", 257)):
        with pytest.raises(rt.RTError, match="RT_ERR_INVALID"):
            rt.set_option(name, bad)
    assert _capi.lib.rt_set_option(99, 0) == -1


def _load_copy(path, tmp_path, name):
    import shutil
    copy = tmp_path / name
    shutil.copyfile(path, copy)
    lib = C.CDLL(str(copy))
    lib.rt_set_option.argtypes = [C.c_int, C.c_int64]
    lib.rt_get_option.argtypes = [C.c_int, C.POINTER(C.c_int64)]
    return lib


def test_product_refuses_tune_bits_that_leave_parity(rt, tmp_path):
    # The product library honours only RT_OPT_TUNE bits that keep the image bits (instance choice,
    # block order, replay-pass form, exact shortcuts off, leaf postponement's q): the inexact
    # prune-all experiment (bit 20), the audit's estimate shrink (bit 29), the ablation bits (8-12),
    # the A/B block-stride bit (23) and the unused kModeExact bit 0 are RT_ERR_INVALID there, and
    # the option keeps its previous value. The audit build (the diagnostic library) still takes its bits.
    from raytracinginoneweekendinrust_amd import _capi
    lib = _load_copy(_capi.LIB_PATH, tmp_path, "librtamd_product_copy.so")
    tune = _capi.OPTIONS["tune"]
    val = C.c_int64(-1)
    for bit in (0, 8, 9, 10, 11, 12, 20, 23, 29, 30, 31):
        assert lib.rt_set_option(tune, 1 << bit) == -1, bit  # RT_ERR_INVALID
        assert lib.rt_get_option(tune, C.byref(val)) == 0 and val.value == 0, bit
    for bits in (1 << 1, 1 << 5, 1 << 6, 1 << 7, 1 << 16, 1 << 17, 1 << 21, 1 << 22, 15 << 24, 3 << 24 | 1 << 16):
        assert lib.rt_set_option(tune, bits) == 0, hex(bits)
        assert lib.rt_get_option(tune, C.byref(val)) == 0 and val.value == bits
    assert lib.rt_set_option(tune, 0) == 0
    audit = os.path.join(os.path.dirname(_capi.LIB_PATH), "librtamd_audit.so")
    alib = _load_copy(audit, tmp_path, "librtamd_audit_copy.so")
    for bits in (1 << 20, 1 << 29, 1 << 20 | 1 << 29 | 1 << 21):
        assert alib.rt_set_option(tune, bits) == 0, hex(bits)
    assert alib.rt_set_option(tune, 1 << 8) == -1  # ablation bits: librtamd_ablate.so only
    assert alib.rt_set_option(tune, 0) == 0
    src = open(os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "csrc", "kernel.hip")).read()
    assert "(kPruneAllExpBuild && (mode & kModePruneAllExp))" in src


def test_abi_layouts_match_the_header_and_the_ctypes_mirror(tmp_path):
    # include/rt.h asserts its struct layouts (RT_LAYOUT_ASSERT) on every C / C++ compile; the
    # ctypes mirror and INTEGRATION.md's #[repr(C)] structs must describe the same bytes.
    from raytracinginoneweekendinrust_amd import _capi
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    inc = os.path.join(root, "include")
    src = tmp_path / "layout.c"
    src.write_text('#include "rt.h"\nint main(void) { return 0; }\n')
    for compiler, std in (("gcc", "-std=c11"), ("g++", "-std=c++17")):
        r = subprocess.run([compiler, std, "-fsyntax-only", "-I", inc, "-x", "c" if compiler == "gcc" else "c++",
                            str(src)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    sizes = {"rt_node": 72, "rt_bvh_node": 40, "rt_scene_desc": 64, "rt_camera": 84, "rt_render_params": 64,
             "rt_stats": 24}
    for name, size in sizes.items():
        assert C.sizeof(getattr(_capi, name)) == size, name
    assert _capi.rt_render_params.seed.offset == 24 and _capi.rt_render_params.spp_total.offset == 60
    assert _capi.rt_scene_desc.bvh_nodes.offset == 48 and _capi.rt_node.seed.offset == 64
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    assert "rt_node = 72 B, rt_bvh_node = 40 B, rt_scene_desc = 64 B, rt_camera = 84 B, rt_render_params = 64 B" in doc
