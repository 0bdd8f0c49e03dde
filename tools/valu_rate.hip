// valu_rate.hip — calibration microbenchmark: the wave64 VALU issue peak of one gfx950 SIMD.
//
// bench.py's roofline.valu prices the trace kernel's vector-ALU work against this peak,
// so it is measured, not assumed: every CU runs W waves per SIMD (W = 1, 2, 3, 4, 8), each
// wave issuing long unrolled blocks of one instruction class in inline asm over 8
// independent accumulators (no dependency stalls once W >= 2), for >= 50 ms per dispatch
// timed with hipEvents. Reported per class and W: wall-clock cycles per wave64 instruction
// per SIMD (dispatch time x shader clock / instructions per SIMD; the clock is the
// s_memtime / s_memrealtime ratio of the same waves) and the same at the nominal 2.4 GHz.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip
//   tools/valu_rate                      # every class, every W: one JSON line each
//   tools/valu_rate <class> <W> [ms]     # one dispatch of one class (for rocprofv3 --pmc)
//
// Built and run only by tools/ (calibration), never by the product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

constexpr int kUnroll = 16;  // asm blocks per loop trip (8 instructions each): 128 per trip

typedef float f2 __attribute__((ext_vector_type(2)));

// One asm block: 8 independent instructions of class kOp on a0..a7.
template <int kOp>
__device__ __forceinline__ void block(float& a0, float& a1, float& a2, float& a3, float& a4, float& a5, float& a6,
                                      float& a7, double& d0, double& d1, double& d2, double& d3, double& d4,
                                      double& d5, double& d6, double& d7, f2& p0, f2& p1, f2& p2, f2& p3, f2& p4,
                                      f2& p5, f2& p6, f2& p7, float m, float c, uint64_t mask) {
#define R8(INS, ...)                                                                                         \
    asm volatile(INS " %0, %0, " __VA_ARGS__ "\n\t" INS " %1, %1, " __VA_ARGS__ "\n\t" INS " %2, %2, "      \
                     __VA_ARGS__ "\n\t" INS " %3, %3, " __VA_ARGS__ "\n\t" INS " %4, %4, " __VA_ARGS__       \
                     "\n\t" INS " %5, %5, " __VA_ARGS__ "\n\t" INS " %6, %6, " __VA_ARGS__ "\n\t" INS        \
                     " %7, %7, " __VA_ARGS__                                                                 \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)            \
                 : "v"(m), "v"(c), "s"(mask))
    if constexpr (kOp == 0) R8("v_add_f32", "%8");
    if constexpr (kOp == 1) R8("v_mul_f32", "%8");
    if constexpr (kOp == 2) R8("v_fma_f32", "%8, %9");
    if constexpr (kOp == 3) R8("v_cndmask_b32_e64", "%8, %10");
    if constexpr (kOp == 4) R8("v_max3_f32", "%8, %9");
    if constexpr (kOp == 5)
        asm volatile(
            "v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\t"
            "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_exp_f32 %7, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    if constexpr (kOp == 6)
        asm volatile(
            "v_sqrt_f32 %0, %0\n\tv_sqrt_f32 %1, %1\n\tv_sqrt_f32 %2, %2\n\tv_sqrt_f32 %3, %3\n\t"
            "v_sqrt_f32 %4, %4\n\tv_sqrt_f32 %5, %5\n\tv_sqrt_f32 %6, %6\n\tv_sqrt_f32 %7, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
#undef R8
#define D8(INS, ...)                                                                                         \
    asm volatile(INS " %0, %0, " __VA_ARGS__ "\n\t" INS " %1, %1, " __VA_ARGS__ "\n\t" INS " %2, %2, "      \
                     __VA_ARGS__ "\n\t" INS " %3, %3, " __VA_ARGS__ "\n\t" INS " %4, %4, " __VA_ARGS__       \
                     "\n\t" INS " %5, %5, " __VA_ARGS__ "\n\t" INS " %6, %6, " __VA_ARGS__ "\n\t" INS        \
                     " %7, %7, " __VA_ARGS__                                                                 \
                 : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)            \
                 : "v"((double)m), "v"((double)c))
    if constexpr (kOp == 7) D8("v_fma_f64", "%8, %9");
    if constexpr (kOp == 8) D8("v_add_f64", "%8");
#undef D8
#define P8(INS, ...)                                                                                         \
    asm volatile(INS " %0, %0, " __VA_ARGS__ "\n\t" INS " %1, %1, " __VA_ARGS__ "\n\t" INS " %2, %2, "      \
                     __VA_ARGS__ "\n\t" INS " %3, %3, " __VA_ARGS__ "\n\t" INS " %4, %4, " __VA_ARGS__       \
                     "\n\t" INS " %5, %5, " __VA_ARGS__ "\n\t" INS " %6, %6, " __VA_ARGS__ "\n\t" INS        \
                     " %7, %7, " __VA_ARGS__                                                                 \
                 : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7)            \
                 : "v"(f2{m, m}), "v"(f2{c, c}))
    if constexpr (kOp == 9) P8("v_pk_add_f32", "%8");
    if constexpr (kOp == 10) P8("v_pk_fma_f32", "%8, %9");
#undef P8
}

constexpr int kOps = 11;
const char* kNames[kOps] = {"v_add_f32",  "v_mul_f32", "v_fma_f32", "v_cndmask_b32", "v_max3_f32",  "v_exp_f32",
                            "v_sqrt_f32", "v_fma_f64", "v_add_f64", "v_pk_add_f32",  "v_pk_fma_f32"};

template <int kOp>
__global__ __launch_bounds__(64) void burn(float* out, float m, float c, uint64_t* clk, int iters) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
    f2 p0{a0, a1}, p1{a1, a2}, p2{a2, a3}, p3{a3, a4}, p4{a4, a5}, p5{a5, a6}, p6{a6, a7}, p7{a7, a0};
    const uint64_t mask = 0x5555555555555555ull;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
            block<kOp>(a0, a1, a2, a3, a4, a5, a6, a7, d0, d1, d2, d3, d4, d5, d6, d7, p0, p1, p2, p3, p4, p5, p6,
                       p7, m, c, mask);
    }
    const float s = (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7) + (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) +
                    (p0.x + p1.x + p2.x + p3.x + p4.x + p5.x + p6.x + p7.x);
    out[blockIdx.x * 64u + threadIdx.x] = s;
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;  // 100 MHz ticks
    }
}

using Kern = void (*)(float*, float, float, uint64_t*, int);
Kern kern(int op) {
    switch (op) {
        case 0: return burn<0>;
        case 1: return burn<1>;
        case 2: return burn<2>;
        case 3: return burn<3>;
        case 4: return burn<4>;
        case 5: return burn<5>;
        case 6: return burn<6>;
        case 7: return burn<7>;
        case 8: return burn<8>;
        case 9: return burn<9>;
        default: return burn<10>;
    }
}

struct Result {
    double ms, ghz;
};

Result dispatch(int op, int blocks, int iters, float* out, uint64_t* clk) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern(op), dim3(blocks), dim3(64), 0, 0, out, 0.999f, 0.5f, clk, iters);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    // shader clock: s_memtime cycles over s_memrealtime (100 MHz) ticks, median of sampled waves
    const int n = blocks < 64 ? blocks : 64;
    uint64_t h[128];
    CHECK(hipMemcpy(h, clk, sizeof(uint64_t) * 2 * n, hipMemcpyDeviceToHost));
    double g[64];
    for (int i = 0; i < n; ++i) g[i] = h[2 * i + 1] ? (double)h[2 * i] / (double)h[2 * i + 1] * 0.1 : 0.0;
    for (int i = 1; i < n; ++i)
        for (int j = i; j > 0 && g[j] < g[j - 1]; --j) {
            double t = g[j];
            g[j] = g[j - 1];
            g[j - 1] = t;
        }
    return Result{ms, g[n / 2]};
}

int main(int argc, char** argv) {
    int cus = 0, simds_per_cu = 4;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int max_blocks = cus * simds_per_cu * 8;
    float* out;
    uint64_t* clk;
    CHECK(hipMalloc(&out, sizeof(float) * 64 * max_blocks));
    CHECK(hipMalloc(&clk, 2 * sizeof(uint64_t) * max_blocks));
    const int insts_per_trip = kUnroll * 8;
    auto measure = [&](int op, int wps, double target_ms, bool print) {
        const int blocks = cus * simds_per_cu * wps;
        // size the dispatch from a short probe so that it lasts about target_ms
        int iters = 256;
        Result r = dispatch(op, blocks, iters, out, clk);
        while (r.ms < 5.0) {
            iters *= 4;
            r = dispatch(op, blocks, iters, out, clk);
        }
        iters = (int)((double)iters * target_ms / r.ms) + 1;
        r = dispatch(op, blocks, iters, out, clk);
        const double simd_insts = (double)insts_per_trip * iters * wps;  // per SIMD
        const double cyc = r.ms * 1e-3 * r.ghz * 1e9 / simd_insts;
        const double cyc24 = r.ms * 1e-3 * 2.4e9 / simd_insts;
        if (print)
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"iters\": %d, \"clock_ghz\": %.3f, "
                   "\"cycles_per_wave64_inst_per_simd\": %.3f, \"cycles_at_2p4ghz\": %.3f, \"cus\": %d}\n",
                   kNames[op], wps, r.ms, iters, r.ghz, cyc, cyc24, cus);
        fflush(stdout);
    };
    if (argc >= 3) {  // one class, one occupancy (the PMC pass)
        int op = -1;
        for (int i = 0; i < kOps; ++i)
            if (!strcmp(argv[1], kNames[i])) op = i;
        if (op < 0) {
            fprintf(stderr, "unknown class %s\n", argv[1]);
            return 2;
        }
        measure(op, atoi(argv[2]), argc > 3 ? atof(argv[3]) : 60.0, true);
    } else {
        const int wps_list[] = {1, 2, 3, 4, 8};
        for (int op = 0; op < kOps; ++op)
            for (int w : wps_list) measure(op, w, 60.0, true);
    }
    CHECK(hipFree(out));
    CHECK(hipFree(clk));
    return 0;
}
