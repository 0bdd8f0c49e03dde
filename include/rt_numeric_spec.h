/*
 * rt_numeric_spec.h — the transcendental functions of the hot path, written
 * once with IEEE-754 basic operations only (+ - * / sqrt floor, comparisons,
 * bit casts) so that the x86-64 host (gcc/clang, SSE2, -ffp-contract=off) and
 * gfx950 (hipcc, -ffp-contract=off, correctly rounded div/sqrt) produce the
 * SAME BITS. This header is a numeric specification shared by the device
 * kernel and the CPU oracle; it contains no rendering logic.
 *
 * Why it exists: the reference calls the platform libm through Rust's
 *   f32::sin  (src/textures/checker.rs:30, src/textures/marble.rs:27,
 *              src/geometry/instance.rs:66)
 *   f32::cos  (src/geometry/instance.rs:67)
 *   f32::tan  (src/camera.rs:57)
 *   f32::acos / f32::atan2 (src/geometry/sphere.rs:42-43)
 *   f32::ln   (src/hittable.rs:209)
 * glibc's float routines are not correctly rounded and have no bit-identical
 * device counterpart. Each rt_* below evaluates in double with a truncation
 * error < 1e-16 relative and rounds once to float, i.e. it returns the
 * correctly rounded result except when the exact value lies within ~1e-16 of a
 * float rounding boundary. tests/test_numeric_spec.py checks every function
 * against Python's math module (<= 1 ulp) on dense input sweeps.
 */
#ifndef RT_NUMERIC_SPEC_H
#define RT_NUMERIC_SPEC_H

#include <stdint.h>

#if defined(__HIP__) || defined(__HIPCC__)
#define RT_SPEC_FN __host__ __device__ static inline __attribute__((always_inline))
#else
#define RT_SPEC_FN static inline
#endif

RT_SPEC_FN uint64_t rt_spec_f64_bits(double x) {
    uint64_t u;
    __builtin_memcpy(&u, &x, sizeof u);
    return u;
}
RT_SPEC_FN double rt_spec_bits_f64(uint64_t u) {
    double x;
    __builtin_memcpy(&x, &u, sizeof x);
    return x;
}
RT_SPEC_FN uint32_t rt_spec_f32_bits(float x) {
    uint32_t u;
    __builtin_memcpy(&u, &x, sizeof u);
    return u;
}
RT_SPEC_FN float rt_spec_bits_f32(uint32_t u) {
    float x;
    __builtin_memcpy(&x, &u, sizeof x);
    return x;
}
RT_SPEC_FN int rt_spec_isnan(double x) { return x != x; }
RT_SPEC_FN double rt_spec_copysign(double mag, double sgn) {
    uint64_t m = rt_spec_f64_bits(mag) & 0x7fffffffffffffffull;
    uint64_t s = rt_spec_f64_bits(sgn) & 0x8000000000000000ull;
    return rt_spec_bits_f64(m | s);
}
RT_SPEC_FN double rt_spec_fabs(double x) {
    return rt_spec_bits_f64(rt_spec_f64_bits(x) & 0x7fffffffffffffffull);
}

#define RT_SPEC_PI 3.141592653589793
#define RT_SPEC_PI_2 1.5707963267948966
#define RT_SPEC_PI_4 0.7853981633974483
#define RT_SPEC_3PI_4 2.356194490192345
#define RT_SPEC_LN2 0.6931471805599453

/* sin(r), cos(r) for |r| <= pi/4: Taylor series to r^15 / r^16 (truncation
 * < 5e-17 relative), Horner in double. */
RT_SPEC_FN double rt_spec_sin_kernel(double r) {
    double z = r * r;
    double p = -1.0 / 1307674368000.0;
    p = 1.0 / 6227020800.0 + z * p;
    p = -1.0 / 39916800.0 + z * p;
    p = 1.0 / 362880.0 + z * p;
    p = -1.0 / 5040.0 + z * p;
    p = 1.0 / 120.0 + z * p;
    p = -1.0 / 6.0 + z * p;
    return r + (r * z) * p;
}
RT_SPEC_FN double rt_spec_cos_kernel(double r) {
    double z = r * r;
    double p = 1.0 / 20922789888000.0;
    p = -1.0 / 87178291200.0 + z * p;
    p = 1.0 / 479001600.0 + z * p;
    p = -1.0 / 3628800.0 + z * p;
    p = 1.0 / 40320.0 + z * p;
    p = -1.0 / 720.0 + z * p;
    p = 1.0 / 24.0 + z * p;
    p = -0.5 + z * p;
    return 1.0 + z * p;
}

/* sin / cos of a double argument with Cody-Waite reduction by pi/2 (fdlibm's
 * 33+33-bit split of pi/2). Accurate for |x| < 1.6e6; deterministic beyond. */
RT_SPEC_FN double rt_spec_sincos_d(double x, int want_cos) {
    if (rt_spec_isnan(x) || rt_spec_fabs(x) == __builtin_inf()) return x - x;
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    double kd = __builtin_floor(x * invpio2 + 0.5);
    if (rt_spec_fabs(kd) > 4503599627370496.0) kd = 0.0; /* |x| > 7e15: keep (int64) defined */
    double r = (x - kd * pio2_1) - kd * pio2_1t;
    int64_t k = (int64_t)kd;
    int q = (int)(k & 3) + (want_cos ? 1 : 0);
    switch (q & 3) {
        case 0: return rt_spec_sin_kernel(r);
        case 1: return rt_spec_cos_kernel(r);
        case 2: return -rt_spec_sin_kernel(r);
        default: return -rt_spec_cos_kernel(r);
    }
}

RT_SPEC_FN float rt_sinf(float x) { return (float)rt_spec_sincos_d((double)x, 0); }
RT_SPEC_FN float rt_cosf(float x) { return (float)rt_spec_sincos_d((double)x, 1); }
RT_SPEC_FN float rt_tanf(float x) {
    double s = rt_spec_sincos_d((double)x, 0);
    double c = rt_spec_sincos_d((double)x, 1);
    return (float)(s / c);
}

/* atan(t) for 0 <= t <= 1: t = c + delta with c = k/8, atan(t) = atan(c) +
 * atan((t-c)/(1+t*c)); |u| <= 1/16 so the odd series to u^13 has truncation
 * < 4e-20. */
RT_SPEC_FN double rt_spec_atan01(double t) {
    double kd = __builtin_floor(t * 8.0 + 0.5);
    int k = (int)kd;
    double c = kd * 0.125;
    double u = (t - c) / (1.0 + t * c);
    double z = u * u;
    double p = -1.0 / 13.0;
    p = 1.0 / 11.0 + z * p;
    p = -1.0 / 9.0 + z * p;
    p = 1.0 / 7.0 + z * p;
    p = -1.0 / 5.0 + z * p;
    p = 1.0 / 3.0 + z * p;
    double a = u - (u * z) * p;
    double base;
    switch (k) {
        case 0: base = 0.0; break;
        case 1: base = 0.12435499454676144; break;
        case 2: base = 0.24497866312686414; break;
        case 3: base = 0.35877067027057225; break;
        case 4: base = 0.4636476090008061; break;
        case 5: base = 0.5585993153435624; break;
        case 6: base = 0.6435011087932844; break;
        case 7: base = 0.7188299996216245; break;
        default: base = 0.7853981633974483; break;
    }
    return base + a;
}

/* atan2 in double with C99 Annex F special cases (signed zeros matter:
 * sphere.rs:43 maps <-1,0,0> to u = 0 through atan2(-0.0, -1) = -pi). */
RT_SPEC_FN double rt_spec_atan2_d(double y, double x) {
    if (rt_spec_isnan(x) || rt_spec_isnan(y)) return x + y;
    double ax = rt_spec_fabs(x), ay = rt_spec_fabs(y);
    int xneg = (rt_spec_f64_bits(x) >> 63) != 0;
    if (ay == 0.0) {
        if (!xneg) return y;                    /* atan2(+-0, +x or +0) = +-0 */
        return rt_spec_copysign(RT_SPEC_PI, y); /* atan2(+-0, -x or -0) = +-pi */
    }
    if (ax == 0.0) return rt_spec_copysign(RT_SPEC_PI_2, y);
    const double inf = __builtin_inf();
    if (ax == inf) {
        if (ay == inf) return rt_spec_copysign(xneg ? RT_SPEC_3PI_4 : RT_SPEC_PI_4, y);
        return xneg ? rt_spec_copysign(RT_SPEC_PI, y) : rt_spec_copysign(0.0, y);
    }
    if (ay == inf) return rt_spec_copysign(RT_SPEC_PI_2, y);
    double a;
    if (ay <= ax) a = rt_spec_atan01(ay / ax);
    else a = RT_SPEC_PI_2 - rt_spec_atan01(ax / ay);
    if (xneg) a = RT_SPEC_PI - a;
    return rt_spec_copysign(a, y);
}

RT_SPEC_FN float rt_atan2f(float y, float x) {
    return (float)rt_spec_atan2_d((double)y, (double)x);
}

/* acos(x) = atan2(sqrt((1-x)(1+x)), x); for float x the product is exact in
 * double and sqrt is correctly rounded on both targets. |x| > 1 -> NaN. */
RT_SPEC_FN float rt_acosf(float xf) {
    double x = (double)xf;
    if (rt_spec_isnan(x)) return xf;
    if (rt_spec_fabs(x) > 1.0) return (float)((x - x) / (x - x)); /* NaN */
    double s = __builtin_sqrt((1.0 - x) * (1.0 + x));
    return (float)rt_spec_atan2_d(s, x);
}

/* ln(x): x = m * 2^e with m in [sqrt(1/2), sqrt(2)); ln(m) = 2 atanh(s),
 * s = (m-1)/(m+1), |s| <= 0.1716, series to s^23 (truncation < 1e-19). */
RT_SPEC_FN double rt_spec_log_d(double x) {
    if (rt_spec_isnan(x)) return x;
    if (x < 0.0) return (x - x) / (x - x);
    if (x == 0.0) return -__builtin_inf();
    if (x == __builtin_inf()) return x;
    uint64_t b = rt_spec_f64_bits(x);
    int e = (int)((b >> 52) & 0x7ff);
    if (e == 0) { /* subnormal double (never from a float argument) */
        x = x * 18014398509481984.0; /* 2^54 */
        b = rt_spec_f64_bits(x);
        e = (int)((b >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    double m = rt_spec_bits_f64((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e += 1;
    }
    double s = (m - 1.0) / (m + 1.0);
    double z = s * s;
    double p = 1.0 / 23.0;
    p = 1.0 / 21.0 + z * p;
    p = 1.0 / 19.0 + z * p;
    p = 1.0 / 17.0 + z * p;
    p = 1.0 / 15.0 + z * p;
    p = 1.0 / 13.0 + z * p;
    p = 1.0 / 11.0 + z * p;
    p = 1.0 / 9.0 + z * p;
    p = 1.0 / 7.0 + z * p;
    p = 1.0 / 5.0 + z * p;
    p = 1.0 / 3.0 + z * p;
    double lnm = 2.0 * s + (2.0 * s * z) * p;
    return (double)e * RT_SPEC_LN2 + lnm;
}

RT_SPEC_FN float rt_logf(float x) { return (float)rt_spec_log_d((double)x); }

/* Rust `f as u32`: saturating, NaN -> 0 (image_texture.rs:28-29). */
RT_SPEC_FN uint32_t rt_f32_to_u32_sat(float x) {
    if (!(x > 0.0f)) return 0u; /* NaN, -0, negatives */
    if (x >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)x;
}

/* Rust f32::to_radians: self * (PI / 180.0) with the quotient folded in f32. */
RT_SPEC_FN float rt_to_radians(float deg) {
    const float k = 3.14159265358979323846f / 180.0f;
    return deg * k;
}

#endif /* RT_NUMERIC_SPEC_H */
