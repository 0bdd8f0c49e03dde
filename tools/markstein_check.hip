// Exhaustive check of the correctly rounded f32 division from a correctly rounded reciprocal
// (Markstein): for y = RN(1/d), q0 = RN(x * y), r = fma(-d, q0, x) (exact), q = RN(q0 + r * y),
// q == RN(x / d) for every pair of f32 significands x, d in [1, 2) (2^46 pairs). Scaling x and d
// by powers of two scales every step exactly while nothing under- or overflows, and signs are
// symmetric, so this covers every input the kernel's gate admits ("Division from the
// hoisted reciprocal"). Also samples the f64 form (y = RN(1/a), a = |d|^2 of an f32 direction) on
// random operands.
//
//   hipcc -O3 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -ffp-contract=off \
//       tools/markstein_check.hip -o /tmp/markstein_check && /tmp/markstein_check [d_blocks]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void check_f32(uint32_t d0, unsigned long long* bad, uint32_t* first) {
    const uint32_t dm = d0 + blockIdx.x;  // d's significand bits
    const float d = __uint_as_float(0x3f800000u | dm);
    const float y = 1.0f / d;  // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
    uint32_t n = 0;
    for (uint32_t xm = threadIdx.x; xm < (1u << 23); xm += 256u) {
        const float x = __uint_as_float(0x3f800000u | xm);
        const float q0 = x * y;
        const float r = __builtin_fmaf(-d, q0, x);
        const float q = __builtin_fmaf(r, y, q0);
        const float ref = x / d;
        if (__float_as_uint(q) != __float_as_uint(ref)) {
            ++n;
            atomicCAS(first, 0xffffffffu, xm);
            atomicCAS(first + 1, 0xffffffffu, dm);
        }
    }
    if (n) atomicAdd(bad, (unsigned long long)n);
}

__device__ __forceinline__ uint64_t mix(uint64_t z) {  // splitmix64
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// f64: a = |d|^2 of a random f32 direction (as to_d computes it), x = a random f64 numerator of
// the sphere roots' magnitude range; q from y = RN(1/a) against RN(x / a).
__global__ __launch_bounds__(256) void check_f64(uint64_t seed, uint32_t per, unsigned long long* bad) {
    uint64_t s = mix(seed ^ ((uint64_t)blockIdx.x << 32 | threadIdx.x));
    uint32_t n = 0;
    for (uint32_t i = 0; i < per; ++i) {
        s = mix(s);
        const float dx = __uint_as_float(0x3f800000u | (uint32_t)(s & 0x7fffffu)) * ((s >> 23) & 1 ? -1.0f : 1.0f);
        const float dy = __uint_as_float(((uint32_t)(s >> 24) & 0x7fffffu) | ((uint32_t)(118u + (s >> 47) % 16u) << 23));
        const float dz = __uint_as_float(((uint32_t)(s >> 32) & 0x7fffffu) | ((uint32_t)(120u + (s >> 51) % 12u) << 23));
        const double a = ((double)dx * dx + (double)dy * dy) + (double)dz * dz;
        s = mix(s);
        const double x = __longlong_as_double((long long)((s & 0x800fffffffffffffull) |
                                                          ((uint64_t)(1023 - 30 + (s >> 52) % 60) << 52)));
        const double y = 1.0 / a;
        const double q0 = x * y;
        const double r = __builtin_fma(-a, q0, x);
        const double q = __builtin_fma(r, y, q0);
        if (__double_as_longlong(q) != __double_as_longlong(x / a)) ++n;
    }
    if (n) atomicAdd(bad, (unsigned long long)n);
}

int main(int argc, char** argv) {
    const uint32_t total = 1u << 23, step = 1u << 15;
    const uint32_t limit = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 0) : total;
    unsigned long long* bad;
    uint32_t* first;
    hipMalloc(&bad, 2 * sizeof(unsigned long long));
    hipMalloc(&first, 2 * sizeof(uint32_t));
    hipMemset(bad, 0, 2 * sizeof(unsigned long long));
    hipMemset(first, 0xff, 2 * sizeof(uint32_t));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (uint32_t d0 = 0; d0 < limit; d0 += step) {
        const uint32_t nb = limit - d0 < step ? limit - d0 : step;
        hipLaunchKernelGGL(check_f32, dim3(nb), dim3(256), 0, 0, d0, bad, first);
        if (((d0 / step) & 31u) == 31u || d0 + nb >= limit) {
            unsigned long long h = 0;
            hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost);
            printf("f32: d significands [0, %u) x all 2^23 x: %llu mismatches\n", d0 + nb, h);
            fflush(stdout);
        }
    }
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h32 = 0;
    uint32_t f[2];
    hipMemcpy(&h32, bad, sizeof h32, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof f, hipMemcpyDeviceToHost);
    printf("f32 exhaustive: %llu pairs, %llu mismatches (first x %#x d %#x), %.1f s\n",
           (unsigned long long)limit << 23, h32, f[0], f[1], ms / 1e3);
    const uint32_t per = 1u << 12, blocks = 1u << 16;
    for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(check_f64, dim3(blocks), dim3(256), 0, 0, (uint64_t)rep * 0x1234567ull + 7, per, bad + 1);
        hipDeviceSynchronize();
        unsigned long long h = 0;
        hipMemcpy(&h, bad + 1, sizeof h, hipMemcpyDeviceToHost);
        printf("f64 random: %llu pairs, %llu mismatches\n", (unsigned long long)(rep + 1) * per * blocks * 256ull, h);
        fflush(stdout);
    }
    return h32 ? 1 : 0;
}
