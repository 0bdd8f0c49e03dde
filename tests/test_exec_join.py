"""Miscompile guard (CPU suite): no vector write may run between a divergent region's
EXEC-narrowing branch target and the EXEC restore of its join (tools/exec_join_check.py).

Round 3's never-executed-code anomaly was this: ROCm 7.2's VGPR allocator split the Rng
buffer's live ranges at the top of the join after start_sample's `if ((d & 3) == 0)
philox_block(...)`, ahead of the join's `s_or_b64 exec, exec, s[..]`, so the two copies
moved r0 / r2 for the lanes that made the call only; the other lanes kept r0 = d and the
next in_unit_sphere() draw was wrong (C1 11834132 segments instead of 11882594). Whether
the allocator split there depended on unrelated code (SLP vectorization, dead blocks,
debug stores), which is why it looked like never-executed code changing results.

librtamd_rngdiv.so (make rngdiv) is kernel.hip built with the per-lane branch
(RT_RNG_UNIFORM=0) under the product's flags: the regression fixture. The checker must
find exactly those copies there and nothing in the product or the audit build.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import exec_join_check as ejc  # noqa: E402
import kernel_resources as kr  # noqa: E402

LIB = os.path.join(ROOT, "raytracinginoneweekendinrust_amd", "_lib")


def test_product_has_no_vector_write_ahead_of_an_exec_restore():
    found = ejc.check_library(kr.DEFAULT_LIB)
    assert not found, [(kr.readable(f), hex(j), w) for f, j, w in found[:10]]


def test_audit_build_is_clean_too():
    path = os.path.join(LIB, "librtamd_audit.so")
    if not os.path.exists(path):
        pytest.skip("audit build absent")
    assert not ejc.check_library(path)


def test_checker_finds_the_rng_buffer_copies_in_the_fixture():
    path = os.path.join(LIB, "librtamd_rngdiv.so")
    assert os.path.exists(path), "make -C raytracinginoneweekendinrust_amd/csrc rngdiv (__graft_entry__.build())"
    found = ejc.check_library(path)
    per = {}
    for fn, join, what in found:
        per.setdefault(kr.readable(fn), []).append(what.split(": ", 1)[1])
    # the BVH-only (C1) and triangle (C4) instances of kernel.hip, where philox_block is a call:
    # two v_mov copies each, r0 and r2 of the buffer, at the join of the time draw's block fetch
    assert set(per) == {"trace_samples<0, 3, 1>", "trace_samples<0, 3, 75>"}, per
    for inst, ops in per.items():
        assert len(ops) == 2 and all(o.startswith("v_mov_b32") for o in ops), (inst, ops)


def test_classifier_on_synthetic_lines():
    ins = ejc.parse("\n".join([
        "0000000000000000 <k>:",
        "\ts_and_saveexec_b64 s[14:15], vcc                          // 000000000000: BE8E206A",
        "\ts_cbranch_execz 2                                           // 000000000004: BF880002",
        "\tv_mov_b32_e32 v1, v2                                        // 000000000008: 7E020302",
        "\tv_add_u32_e32 v3, 1, v3                                     // 00000000000C: 68060681",
        "\tv_mov_b32_e32 v4, v2                                        // 000000000010: 7E080302",
        "\ts_or_b64 exec, exec, s[14:15]                               // 000000000014: 87FE0E7E",
    ]))
    assert [m for _, _, m, _ in ins] == ["s_and_saveexec_b64", "s_cbranch_execz", "v_mov_b32_e32", "v_add_u32_e32",
                                         "v_mov_b32_e32", "s_or_b64"]
    assert ejc.narrows_exec("s_and_saveexec_b64", "s[14:15], vcc")
    assert not ejc.narrows_exec("s_or_b64", "exec, exec, s[14:15]")
    assert ejc.writes_exec("s_or_b64", "exec, exec, s[14:15]")
    assert ejc.writes_vgpr("v_mov_b32_e32", "v4, v2") and not ejc.writes_vgpr("v_readlane_b32", "s0, v142, 3")
    assert not ejc.writes_vgpr("v_cmp_eq_u32_e32", "vcc, 0, v1")
