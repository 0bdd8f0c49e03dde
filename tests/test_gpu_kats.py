"""The reference's own unit tests and doc-comment known answers, run on the DEVICE
through the kernel's own primitives (rt_device_kat), not only on the oracle:

  src/aabb.rs:73-97    Aabb::hit `hits` / `misses` — exact slab test (op 0) and, for the
                       rays the fast kernel traverses (finite non-zero 1/d), the packed
                       four-child test (op 1)
  src/geometry/sphere.rs:37-40   Sphere::get_uv's six examples (op 2)

plus dense random cases against the oracle restatement bit for bit (aabb_hit for the
boxes, the uv formulas) and the fast test against the exact one. (aabb.rs:99-140, the
union tests, exercise host code the device never runs: test_reference_units.py.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_aabb_rs_hits_and_misses_on_device(rt):  # aabb.rs:73-97
    hits = [-1, -1, 1, 1, 1, 2, 0, 0, 0, 0, 0, 1, 0.0, 5.0]
    misses = [1, 1, 1, 2, 2, 2, 0, 0, 0, 0, 0, 1, 0.0, 5.0]
    r = rt.device_kat(0, [hits, misses])
    assert r[0, 0] == 1.0 and r[1, 0] == 0.0


def test_aabb_rs_cases_through_the_fast_box_test(rt):
    # the same boxes, rays tilted off the axes (the fast kernel only takes rays with
    # 0 < |1/d| < inf on every axis; the axis-parallel ones go to the exact kernel)
    hits = [-1, -1, 1, 1, 1, 2, 0, 0, 0, 1e-3, 1e-3, 1, 0.0, 5.0]
    misses = [1, 1, 1, 2, 2, 2, 0, 0, 0, 1e-3, 1e-3, 1, 0.0, 5.0]
    r = rt.device_kat(1, [hits, misses])
    assert r[0, 0] == 1.0 and r[1, 0] == 0.0


@pytest.mark.parametrize("p,uv", [((1, 0, 0), (0.5, 0.5)), ((-1, 0, 0), (0.0, 0.5)), ((0, 1, 0), (0.5, 1.0)),
                                   ((0, -1, 0), (0.5, 0.0)), ((0, 0, 1), (0.25, 0.5)), ((0, 0, -1), (0.75, 0.5))])
def test_sphere_rs_get_uv_examples_on_device(rt, orc, p, uv):  # sphere.rs:37-40
    got = rt.device_kat(2, [p])[0]
    assert got[0] == pytest.approx(uv[0], abs=1e-6) and got[1] == pytest.approx(uv[1], abs=1e-6)
    np.testing.assert_array_equal(got, np.array(orc.sphere_uv(p), dtype=np.float32))


def test_zero_direction_components_fast_equals_exact(rt, orc):
    # The fast test on rays with exactly zero (+0 / -0) direction components (1/d = +-inf), as the
    # triangle-only BVHs take them since round 6 (kernel.hip ray_route): slab values are +-inf, or
    # 0 * inf = NaN where the origin lies on a slab plane, which aabb.rs:28-41's comparisons ignore
    # and max / min ignore too. aabb.rs:73-97's boxes with the axis-parallel rays of its own tests,
    # then random boxes whose planes the origins sit on; hit flag and entry equal the exact test's,
    # and both equal the oracle's restatement of aabb.rs.
    rng = np.random.default_rng(17)
    cases = [[-1, -1, 1, 1, 1, 2, 0, 0, 0, 0, 0, 1, 0.0, 5.0], [1, 1, 1, 2, 2, 2, 0, 0, 0, 0, 0, 1, 0.0, 5.0],
             [-1, -1, 1, 1, 1, 2, 0, 0, 0, -0.0, 0.0, 1, 0.0, 5.0], [-1, -1, 1, 1, 1, 2, 1, 1, 0, 0, 0, 1, 0.0, 5.0],
             [-1, -1, 1, 1, 1, 2, 1, -1, 0, 0, -0.0, 1, 0.0, float("inf")]]
    n = 6000
    mn = rng.integers(-8, 8, (n, 3)).astype(np.float32)
    mx = mn + rng.integers(0, 5, (n, 3)).astype(np.float32)
    o = rng.integers(-10, 10, (n, 3)).astype(np.float32)
    pick = rng.integers(0, 3, (n, 3))  # origin coordinates on the min plane, the max plane or elsewhere
    o = np.where(pick == 0, mn, np.where(pick == 1, mx, o)).astype(np.float32)
    d = ((mn + mx) / 2 - o + rng.normal(scale=1.0, size=(n, 3))).astype(np.float32)
    zero = rng.random((n, 3)) < 0.45
    sign = rng.random((n, 3)) < 0.5
    d = np.where(zero, np.where(sign, np.float32(-0.0), np.float32(0.0)), d).astype(np.float32)
    zero[:, 0] |= ~zero.any(axis=1)  # at least one zero component per ray
    d[:, 0] = np.where(zero[:, 0] & (d[:, 0] != 0), np.float32(0.0), d[:, 0])
    t = np.stack([rng.uniform(0, 0.3, n), np.where(rng.random(n) < 0.3, np.inf, rng.uniform(0.5, 30, n))],
                 axis=1).astype(np.float32)
    cases = np.concatenate([np.array(cases, dtype=np.float32), np.concatenate([mn, mx, o, d, t], axis=1)])
    exact = rt.device_kat(0, cases)
    fast = rt.device_kat(1, cases)
    want = np.array([orc.aabb_hit(c[0:3], c[3:6], c[6:9], c[9:12], c[12], c[13]) for c in cases])
    assert exact[0, 0] == 1.0 and exact[1, 0] == 0.0  # aabb.rs:73-97 hits / misses
    np.testing.assert_array_equal(exact[:, 0] == 1.0, want)
    np.testing.assert_array_equal(fast[:, 0], exact[:, 0])
    hit = exact[:, 0] == 1.0
    assert 0.1 < hit.mean() < 0.9, hit.mean()
    np.testing.assert_array_equal(fast[hit, 1], np.minimum(exact[hit, 1], np.float32(3.4028235e38)))


def test_random_boxes_device_equals_oracle_and_fast_equals_exact(rt, orc):
    rng = np.random.default_rng(9)
    n = 20000
    mn = rng.uniform(-10, 10, (n, 3)).astype(np.float32)
    mx = mn + rng.uniform(0, 5, (n, 3)).astype(np.float32)
    o = rng.uniform(-15, 15, (n, 3)).astype(np.float32)
    # aimed near the box so that about half the rays hit
    d = ((mn + mx) / 2 - o + rng.normal(scale=1.0, size=(n, 3))).astype(np.float32)
    t = np.stack([rng.uniform(0, 0.3, n), rng.uniform(0.5, 3, n)], axis=1).astype(np.float32)
    cases = np.concatenate([mn, mx, o, d, t], axis=1)
    exact = rt.device_kat(0, cases)
    fast = rt.device_kat(1, cases)
    want = np.array([orc.aabb_hit(c[0:3], c[3:6], c[6:9], c[9:12], c[12], c[13]) for c in cases[:4000]])
    np.testing.assert_array_equal(exact[:4000, 0] == 1.0, want)
    np.testing.assert_array_equal(fast[:, 0], exact[:, 0])
    hit = exact[:, 0] == 1.0
    assert 0.2 < hit.mean() < 0.9, hit.mean()
    np.testing.assert_array_equal(fast[hit, 1], np.minimum(exact[hit, 1], np.float32(3.4028235e38)))


def test_random_sphere_uv_device_equals_oracle(rt, orc):
    rng = np.random.default_rng(4)
    p = rng.normal(size=(3000, 3))
    p = (p / np.linalg.norm(p, axis=1, keepdims=True)).astype(np.float32)
    got = rt.device_kat(2, p)
    want = np.array([orc.sphere_uv(q) for q in p], dtype=np.float32)
    np.testing.assert_array_equal(got, want)


def test_cube_side_quotient_from_the_reciprocal_is_the_division(rt):
    # A BVH cube leaf forms each side's t = (k - o) / d from the ray's reciprocal RN(1/d) and Markstein's
    # correction when k, o and d are in range (kernel.hip rcp_quotient / rcp_ray_ok), the division
    # otherwise. The exhaustive significand check is tools/markstein_check.hip
    # (profiles/r05/markstein_check.log); here random in-range operands over the whole gate, its edges
    # and the special values, against numpy's correctly rounded f32 arithmetic, bit for bit.
    rng = np.random.default_rng(11)
    n = 1 << 20

    def ranged(size, lo=-20, hi=20):
        e = rng.integers(127 + lo, 127 + hi, size=size, dtype=np.uint32)
        m = rng.integers(0, 1 << 23, size=size, dtype=np.uint32)
        v = ((e << 23) | m).view(np.float32)
        return v * np.where(rng.random(size) < 0.5, -1, 1).astype(np.float32)

    cases = [np.stack([ranged(n), ranged(n), ranged(n)], axis=1)]
    # near-equal k and o (cancellation), zeros, and operands just outside the gate
    k = ranged(n)
    o = (k.astype(np.float64) * (1 + rng.normal(0, 1e-6, n))).astype(np.float32)
    cases.append(np.stack([k, o, ranged(n)], axis=1))
    edge = np.array([0.0, -0.0, 2.0 ** -20, -(2.0 ** -20), 2.0 ** 20, 2.0 ** -21, 2.0 ** 21, 1e-45, 3e38, np.inf,
                     np.nan, 1.0, -1.0, 3.0, 0.1, 555.0, 1e-7], dtype=np.float32)
    g = np.array(np.meshgrid(edge, edge, edge)).reshape(3, -1).T
    cases.append(g.astype(np.float32))
    a = np.concatenate(cases).astype(np.float32)
    out = rt.device_kat(4, a)
    with np.errstate(all="ignore"):
        want = ((a[:, 0] - a[:, 1]) / a[:, 2]).astype(np.float32)
    for col in (1, 0):  # the device's own division, then the reciprocal form, against the host
        got = out[:, col]
        same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
        assert same.all(), (col, a[~same][:5], got[~same][:5], want[~same][:5])
