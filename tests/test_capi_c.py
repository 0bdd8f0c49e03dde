"""The drop-in boundary from C: tests/capi/prebuilt_tree.c (compiled by build(),
not ctypes) uploads RT_OBJ_BVH_TREE trees built by the caller and renders with an
explicit Camera (rt_camera, src/camera.rs:6-27) through rt_render_camera; the
program itself compares the image and segment count with oracle_render_camera
fed the same descriptor, bit for bit, and exits non-zero on any difference."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "capi", "_build", "prebuilt_tree")


@pytest.mark.gpu
def test_c_program_prebuilt_tree_and_camera_basis_bit_exact():
    assert os.path.exists(BIN), "build() compiles tests/capi/prebuilt_tree.c"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


def test_c_program_is_built():
    assert os.path.exists(BIN), "build() compiles tests/capi/prebuilt_tree.c"
