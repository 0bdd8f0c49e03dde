// valu_rate.hip — calibration microbenchmark: wave64 VALU throughput per SIMD on gfx950.
//
// The trace kernel's roofline is vector-ALU issue (bench.py roofline.valu), so the
// cycles one wave64 VALU instruction occupies a SIMD must be known: this runs long
// chains of independent f32 FMAs / f64 FMAs / packed f32 FMAs / f32 adds at 1..8
// waves per SIMD on every CU and reports instructions per SIMD-cycle (clock from
// s_memtime deltas vs wall time). Built and run only by tools/ (not the product).
//
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

static int kIters = 4096;  // argv[1] overrides (longer runs for the PMC calibration pass)
constexpr int kChains = 8;  // independent accumulators: enough ILP for one wave

template <int kOp>
__global__ void burn(float* out, float a, float b, uint64_t* clk, int iters) {
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (kOp == 0 || kOp == 3) {  // v_fma_f32 / v_add_f32
        float x[kChains];
#pragma unroll
        for (int c = 0; c < kChains; ++c) x[c] = threadIdx.x * 1e-3f + c;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int c = 0; c < kChains; ++c) {
                if constexpr (kOp == 0) x[c] = __builtin_fmaf(x[c], a, b);
                else x[c] = x[c] + a;
            }
        }
        float s = 0.0f;
#pragma unroll
        for (int c = 0; c < kChains; ++c) s += x[c];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    } else if constexpr (kOp == 1) {  // v_fma_f64
        double x[kChains];
#pragma unroll
        for (int c = 0; c < kChains; ++c) x[c] = threadIdx.x * 1e-3 + c;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int c = 0; c < kChains; ++c) x[c] = __builtin_fma(x[c], (double)a, (double)b);
        }
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < kChains; ++c) s += x[c];
        out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
    } else {  // v_pk_fma_f32
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 x[kChains / 2];
        const f2 av = {a, a}, bv = {b, b};
#pragma unroll
        for (int c = 0; c < kChains / 2; ++c) x[c] = f2{threadIdx.x * 1e-3f + c, (float)c};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int c = 0; c < kChains / 2; ++c) x[c] = __builtin_elementwise_fma(x[c], av, bv);
        }
        float s = 0.0f;
#pragma unroll
        for (int c = 0; c < kChains / 2; ++c) s += x[c].x + x[c].y;
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;  // 100 MHz ticks
    }
}

template <int kOp>
void run(const char* name, int cus) {
    float* out;
    uint64_t* clk;
    const int max_blocks = cus * 32;
    hipMalloc(&out, sizeof(float) * 64 * max_blocks);
    hipMalloc(&clk, 2 * sizeof(uint64_t) * max_blocks);
    const int insts_per_wave = kIters * (kOp == 2 ? kChains / 2 : kChains);
    for (int wps = 1; wps <= 8; wps *= 2) {  // waves per SIMD
        const int blocks = cus * 4 * wps;      // 64-thread blocks, spread over all SIMDs
        hipLaunchKernelGGL(burn<kOp>, dim3(blocks), dim3(64), 0, 0, out, 1.0001f, 0.5f, clk, kIters);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        const int reps = 5;
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(burn<kOp>, dim3(blocks), dim3(64), 0, 0, out, 1.0001f, 0.5f, clk, kIters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        uint64_t c2[2] = {0, 0};
        hipMemcpy(c2, clk, sizeof c2, hipMemcpyDeviceToHost);
        const uint64_t c0 = c2[0];
        const double ghz = c2[1] ? (double)c2[0] / (double)c2[1] * 0.1 : 0.0;  // s_memtime rate vs 100 MHz
        // instructions per SIMD per cycle, with the clock taken from one wave's s_memtime span
        const double s = ms / 1e3 / reps;
        const double simd_inst = (double)insts_per_wave * wps;  // per SIMD per launch
        const double cyc_wave = (double)c0;
        printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_inst_per_simd\": %.3f, "
               "\"cycles_per_inst_one_wave\": %.3f, \"memtime_ghz\": %.3f, \"ns_per_inst_one_wave\": %.4f}\n",
               name, wps, s * 1e3, cyc_wave / simd_inst, cyc_wave / insts_per_wave, ghz,
               ghz > 0 ? cyc_wave / ghz / insts_per_wave : 0.0);
        hipEventDestroy(e0);
        hipEventDestroy(e1);
    }
    hipFree(out);
    hipFree(clk);
}

int main(int argc, char** argv) {
    if (argc > 1) kIters = atoi(argv[1]);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("{\"cus\": %d}\n", cus);
    run<0>("v_fma_f32", cus);
    run<3>("v_add_f32", cus);
    run<1>("v_fma_f64", cus);
    run<2>("v_pk_fma_f32", cus);
    return 0;
}
