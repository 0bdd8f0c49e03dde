// bvh_build.hip — Bvh::new's split order on the device.
//
// BvhNode::new_helper (src/bvh.rs:249-333) draws a random axis per node, stable-sorts
// the node's items by bounding_box(0, 0).min[axis] (total_cmp, :420-440), splits at
// n / 2 and recurses; two-item nodes order their pair with one comparison (:270-281,
// an unsorted swap: equal keys DO swap), one-item nodes hold the item twice. The
// tree's shape depends on n alone and the axes on the seed alone, so the host lays
// out the schedule (bvh_split_schedule: every node's start, count and axis, by
// depth) and the device produces the only key-dependent output, the final leaf
// order, level by level:
//
//   level_keys   composite 64-bit key per position: (start of its node << 32) |
//                total-order bits of key[axis] for nodes of > 2 items; positions of
//                finished leaves get (position << 32), which keeps them in place
//   radix sort   rocPRIM radix_sort_pairs over (key, item) — stable, so equal keys
//                keep the order the parent's sort left, as the stable merge sort does
//   pair_order   the two-item leaves' single comparison, applied once at the end
//                (leaves are never touched by a deeper level)
//
// One sort of n pairs per level, log2(n) + 1 levels; the host recursion does the
// same n log n work per level in a single thread.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <string>
#include <vector>

#include "../../include/rt.h"
#include "common.hpp"
#include "lower.hpp"

namespace {

// f32 total_cmp order as an unsigned key (Rust f32::total_cmp: -NaN < -inf < ... < -0 < +0 < ... < +NaN).
__device__ __forceinline__ uint32_t total_order_bits(float f) {
    const uint32_t u = __float_as_uint(f);
    return u ^ ((u >> 31) ? 0xFFFFFFFFu : 0x80000000u);
}

// i = position in the current order. Nodes of level L (sorted by start, > 2 items
// only) are [seg, seg + nseg).
__global__ __launch_bounds__(256) void level_keys(const float* __restrict__ keys, const uint32_t* __restrict__ order,
                                                  const uint32_t* __restrict__ start, const uint32_t* __restrict__ count,
                                                  const uint32_t* __restrict__ axis, uint32_t nseg, uint32_t n,
                                                  uint64_t* __restrict__ out) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        uint32_t lo = 0, hi = nseg;  // last node with start <= i
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (start[m] <= i) lo = m + 1;
            else hi = m;
        }
        uint64_t k = (uint64_t)i << 32;
        if (lo > 0) {
            const uint32_t j = lo - 1, s = start[j];
            if (i - s < count[j]) k = ((uint64_t)s << 32) | total_order_bits(keys[3u * order[i] + axis[j]]);
        }
        out[i] = k;
    }
}

__global__ void iota(uint32_t* __restrict__ order, uint32_t n) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) order[i] = i;
}

// bvh.rs:270-281: (objects[0], objects[1]) if compare(0, 1) == Less, else swapped.
__global__ void pair_order(const float* __restrict__ keys, uint32_t* __restrict__ order,
                           const uint32_t* __restrict__ start, const uint32_t* __restrict__ axis, uint32_t m) {
    for (uint32_t k = blockIdx.x * 256u + threadIdx.x; k < m; k += gridDim.x * 256u) {
        const uint32_t s = start[k], a = order[s], b = order[s + 1u], ax = axis[k];
        if (!(total_order_bits(keys[3u * a + ax]) < total_order_bits(keys[3u * b + ax]))) {
            order[s] = b;
            order[s + 1u] = a;
        }
    }
}

uint32_t grid_for(uint64_t n) {
    uint64_t g = (n + 255u) / 256u;
    return (uint32_t)(g < 4096u ? (g ? g : 1u) : 4096u);
}

uint32_t bits_for(uint32_t v) {  // bits to hold 0..v
    uint32_t b = 0;
    while (b < 32u && (v >> b)) ++b;
    return b;
}

struct DevBufs {
    std::vector<void*> p;
    ~DevBufs() {
        for (void* x : p)
            if (x) (void)hipFree(x);
    }
    template <class T>
    hipError_t alloc(T** out, size_t n) {
        void* x = nullptr;
        hipError_t e = hipMalloc(&x, n ? n * sizeof(T) : 1);
        if (e == hipSuccess) p.push_back(x);
        *out = (T*)x;
        return e;
    }
};

}  // namespace

extern "C" int rt_bvh_build_order(const float* d_keys, uint32_t n, uint64_t seed, uint32_t* d_order, void* stream) {
    rthost::clear_error();
    if (n && (!d_keys || !d_order)) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    if (n >= 0x80000000u) return rthost::set_error(RT_ERR_INVALID, "more than 2^31 - 1 items");
    if (n == 0) return RT_OK;
    hipStream_t st = (hipStream_t)stream;
    rthost::BvhSchedule sc;
    rthost::bvh_split_schedule(n, seed, &sc);
    // Split the schedule into the sorted nodes (> 2 items) per level and the pair leaves.
    std::vector<uint32_t> s_start, s_count, s_axis, lvl{0}, p_start, p_axis;
    for (size_t L = 0; L + 1 < sc.level_off.size(); ++L) {
        for (uint32_t j = sc.level_off[L]; j < sc.level_off[L + 1]; ++j) {
            if (sc.count[j] > 2) {
                s_start.push_back(sc.start[j]);
                s_count.push_back(sc.count[j]);
                s_axis.push_back(sc.axis[j]);
            } else if (sc.count[j] == 2) {
                p_start.push_back(sc.start[j]);
                p_axis.push_back(sc.axis[j]);
            }
        }
        lvl.push_back((uint32_t)s_start.size());
    }
    DevBufs b;
    uint32_t *ds = nullptr, *dc = nullptr, *da = nullptr, *dps = nullptr, *dpa = nullptr, *alt = nullptr;
    uint64_t *k0 = nullptr, *k1 = nullptr;
    hipError_t e;
    if ((e = b.alloc(&ds, s_start.size())) || (e = b.alloc(&dc, s_count.size())) || (e = b.alloc(&da, s_axis.size())) ||
        (e = b.alloc(&dps, p_start.size())) || (e = b.alloc(&dpa, p_axis.size())) || (e = b.alloc(&alt, n)) ||
        (e = b.alloc(&k0, n)) || (e = b.alloc(&k1, n)))
        return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc (BVH build): ") + hipGetErrorString(e));
    auto h2d = [&](void* dst, const std::vector<uint32_t>& v) {
        return v.empty() ? hipSuccess : hipMemcpyAsync(dst, v.data(), v.size() * 4u, hipMemcpyHostToDevice, st);
    };
    if ((e = h2d(ds, s_start)) || (e = h2d(dc, s_count)) || (e = h2d(da, s_axis)) || (e = h2d(dps, p_start)) ||
        (e = h2d(dpa, p_axis)))
        return rthost::set_error(RT_ERR_HIP, std::string("BVH schedule upload: ") + hipGetErrorString(e));
    const uint32_t end_bit = 32u + bits_for(n - 1u);
    size_t tmp_bytes = 0;
    if ((e = rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, d_order, alt, (size_t)n, 0u, end_bit, st)))
        return rthost::set_error(RT_ERR_HIP, std::string("radix sort query: ") + hipGetErrorString(e));
    uint8_t* tmp = nullptr;
    if ((e = b.alloc(&tmp, tmp_bytes)))
        return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc (sort scratch): ") + hipGetErrorString(e));
    (void)hipGetLastError();
    uint32_t* cur = d_order;
    uint32_t* nxt = alt;
    hipLaunchKernelGGL(iota, dim3(grid_for(n)), dim3(256), 0, st, cur, n);
    for (size_t L = 0; L + 1 < lvl.size(); ++L) {
        const uint32_t nseg = lvl[L + 1] - lvl[L];
        if (!nseg) continue;
        hipLaunchKernelGGL(level_keys, dim3(grid_for(n)), dim3(256), 0, st, d_keys, cur, ds + lvl[L], dc + lvl[L],
                           da + lvl[L], nseg, n, k0);
        if ((e = rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, cur, nxt, (size_t)n, 0u, end_bit, st)))
            return rthost::set_error(RT_ERR_HIP, std::string("radix sort: ") + hipGetErrorString(e));
        std::swap(cur, nxt);
    }
    if (!p_start.empty())
        hipLaunchKernelGGL(pair_order, dim3(grid_for(p_start.size())), dim3(256), 0, st, d_keys, cur, dps, dpa,
                           (uint32_t)p_start.size());
    if (cur != d_order && (e = hipMemcpyAsync(d_order, cur, (size_t)n * 4u, hipMemcpyDeviceToDevice, st)))
        return rthost::set_error(RT_ERR_HIP, std::string("BVH order copy: ") + hipGetErrorString(e));
    if ((e = hipGetLastError()) || (e = hipStreamSynchronize(st)))
        return rthost::set_error(RT_ERR_HIP, std::string("BVH build: ") + hipGetErrorString(e));
    return RT_OK;
}

namespace rthost {

// BvhOrderer::fn for rt_scene_upload: ctx points at the target device id.
int device_bvh_order(void* ctx, const float* keys, uint32_t n, uint64_t seed, uint32_t* order, std::string* err) {
    const int device = *(const int*)ctx;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    struct Restore {
        int prev;
        ~Restore() {
            if (prev >= 0) (void)hipSetDevice(prev);
        }
    } restore{prev};
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        *err = std::string("BVH build on device ") + std::to_string(device) + ": " + hipGetErrorString(e);
        return RT_ERR_NO_DEVICE;
    }
    DevBufs b;
    float* dk = nullptr;
    uint32_t* dord = nullptr;
    hipStream_t st = nullptr;
    if ((e = b.alloc(&dk, 3u * (size_t)n)) || (e = b.alloc(&dord, n))) {
        *err = std::string("hipMalloc (BVH build): ") + hipGetErrorString(e);
        return RT_ERR_OOM;
    }
    if ((e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking))) {
        *err = std::string("hipStreamCreate: ") + hipGetErrorString(e);
        return RT_ERR_HIP;
    }
    int rc = RT_OK;
    if ((e = hipMemcpyAsync(dk, keys, 12u * (size_t)n, hipMemcpyHostToDevice, st))) {
        rc = RT_ERR_HIP;
        *err = std::string("BVH keys upload: ") + hipGetErrorString(e);
    } else if ((rc = rt_bvh_build_order(dk, n, seed, dord, st))) {
        *err = rt_last_error();
    } else if ((e = hipMemcpyAsync(order, dord, 4u * (size_t)n, hipMemcpyDeviceToHost, st)) ||
               (e = hipStreamSynchronize(st))) {
        rc = RT_ERR_HIP;
        *err = std::string("BVH order download: ") + hipGetErrorString(e);
    }
    (void)hipStreamDestroy(st);
    return rc;
}

}  // namespace rthost
