// output.hip — the output step of Renderer::render on the device.
//
// src/renderer.rs:107-127 writes "P3\nW H\n255\n" and then one "r g b\n" line per
// pixel, rows from the top (y = H-1) down, each channel converted by palette
// 0.6.1 (Srgb<f32> -> Srgb<u8>: clamp to [0, 1] with NaN -> 0, x 255, round half
// away from zero; srgb_from_vec3 applies no gamma, src/utils.rs:19-23). The ASCII
// formatting of W*H lines sits inside the reference's timer. Here it is three
// launches: quantise + per-line length, an exclusive scan of the lengths
// (rocPRIM), and a writer that puts every line at its offset.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_scan.hpp>

#include <string>

#include "../../include/rt.h"
#include "common.hpp"

namespace {

__device__ __forceinline__ uint32_t to_u8(float c) {  // palette 0.6.1 f32 -> u8
    if (!(c > 0.0f)) c = 0.0f;
    if (c > 1.0f) c = 1.0f;
    return (uint32_t)roundf(c * 255.0f);
}
__device__ __forceinline__ uint32_t digits(uint32_t v) { return v >= 100u ? 3u : (v >= 10u ? 2u : 1u); }

// i = output line (rows top to bottom); writes the 3 bytes and the line length.
__global__ __launch_bounds__(256) void quantise_lines(const float* __restrict__ rgb, uint8_t* __restrict__ u8,
                                                      uint64_t* __restrict__ len, uint32_t width, uint32_t height) {
    const uint64_t n = (uint64_t)width * height;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const uint64_t yo = i / width, x = i - yo * width;
        const float* c = rgb + ((height - 1u - yo) * (uint64_t)width + x) * 3u;
        const uint32_t r = to_u8(c[0]), g = to_u8(c[1]), b = to_u8(c[2]);
        u8[3u * i] = (uint8_t)r;
        u8[3u * i + 1u] = (uint8_t)g;
        u8[3u * i + 2u] = (uint8_t)b;
        if (len) len[i] = digits(r) + digits(g) + digits(b) + 3u;
    }
}

__device__ __forceinline__ char* put_u(char* p, uint32_t v) {
    if (v >= 100u) *p++ = (char)('0' + v / 100u);
    if (v >= 10u) *p++ = (char)('0' + (v / 10u) % 10u);
    *p++ = (char)('0' + v % 10u);
    return p;
}

__global__ __launch_bounds__(256) void write_lines(const uint8_t* __restrict__ u8, const uint64_t* __restrict__ off,
                                                   char* __restrict__ text, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        char* p = text + off[i];
        p = put_u(p, u8[3u * i]);
        *p++ = ' ';
        p = put_u(p, u8[3u * i + 1u]);
        *p++ = ' ';
        p = put_u(p, u8[3u * i + 2u]);
        *p = '\n';
    }
}

int hip_fail(hipError_t e, const char* what) {
    return rthost::set_error(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

uint32_t grid_for(uint64_t n) {
    uint64_t g = (n + 255u) / 256u;
    return (uint32_t)(g < 65536u ? (g ? g : 1u) : 65536u);
}

}  // namespace

extern "C" {

int rt_quantize_srgb8(const float* d_rgb, uint8_t* d_u8, uint32_t width, uint32_t height, void* stream) {
    rthost::clear_error();
    if (!d_rgb || !d_u8) return rthost::set_error(RT_ERR_INVALID, "NULL buffer");
    const uint64_t n = (uint64_t)width * height;
    if (n == 0) return RT_OK;
    (void)hipGetLastError();  // drop a stale error left by an earlier, unrelated HIP call
    hipLaunchKernelGGL(quantise_lines, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, d_rgb, d_u8,
                       (uint64_t*)nullptr, width, height);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RT_OK : hip_fail(e, "quantise launch");
}

int rt_format_ppm(const float* d_rgb, uint32_t width, uint32_t height, char* d_text, uint64_t capacity,
                  uint64_t* text_bytes, void* stream) {
    rthost::clear_error();
    if (!d_rgb || !d_text || !text_bytes) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    const uint64_t n = (uint64_t)width * height;
    *text_bytes = 0;
    if (n == 0) return RT_OK;
    if (capacity < n * 12u) return rthost::set_error(RT_ERR_INVALID, "text buffer smaller than 12 bytes per pixel");
    hipStream_t st = (hipStream_t)stream;
    uint8_t* u8 = nullptr;
    uint64_t *len = nullptr, *off = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hipError_t e;
    auto cleanup = [&]() {
        if (u8) (void)hipFree(u8);
        if (len) (void)hipFree(len);
        if (off) (void)hipFree(off);
        if (tmp) (void)hipFree(tmp);
    };
    if ((e = hipMalloc(&u8, 3u * n)) != hipSuccess || (e = hipMalloc(&len, 8u * n)) != hipSuccess ||
        (e = hipMalloc(&off, 8u * n)) != hipSuccess) {
        cleanup();
        return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    (void)hipGetLastError();  // as above
    hipLaunchKernelGGL(quantise_lines, dim3(grid_for(n)), dim3(256), 0, st, d_rgb, u8, len, width, height);
    if ((e = hipGetLastError()) != hipSuccess) {
        cleanup();
        return hip_fail(e, "quantise launch");
    }
    if ((e = rocprim::exclusive_scan(nullptr, tmp_bytes, len, off, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(),
                                     st)) != hipSuccess ||
        (e = hipMalloc(&tmp, tmp_bytes ? tmp_bytes : 1)) != hipSuccess ||
        (e = rocprim::exclusive_scan(tmp, tmp_bytes, len, off, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(),
                                     st)) != hipSuccess) {
        cleanup();
        return hip_fail(e, "line offset scan");
    }
    hipLaunchKernelGGL(write_lines, dim3(grid_for(n)), dim3(256), 0, st, u8, off, d_text, n);
    uint64_t last_off = 0, last_len = 0;
    if ((e = hipGetLastError()) != hipSuccess ||
        (e = hipMemcpyAsync(&last_off, off + (n - 1u), 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipMemcpyAsync(&last_len, len + (n - 1u), 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess) {
        cleanup();
        return hip_fail(e, "format ppm");
    }
    *text_bytes = last_off + last_len;
    cleanup();
    return RT_OK;
}

}  // extern "C"
