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
    # kernel.hip's instances that the fixture's allocator split that way: the C1 instance (which
    # tests/test_gpu_exec_join.py renders) among them, two v_mov copies (r0, r2 of the buffer)
    # at the join of the time draw's block fetch in each; which other instances show it moves
    # with unrelated code (round 4: the triangle preset's, later the all-feature ones)
    assert "trace_samples<0, 3, 1>" in per, per
    for inst, ops in per.items():
        assert inst.startswith("trace_samples<0,"), (inst, ops)
        assert len(ops) == 2 and all(o.startswith("v_mov_b32") for o in ops), (inst, ops)
