// bvh_build.hip — Bvh::new's split order on the device.
//
// BvhNode::new_helper (src/bvh.rs:249-333) draws a random axis per node, stable-sorts
// the node's items by bounding_box(0, 0).min[axis] (total_cmp, :420-440), splits at
// n / 2 and recurses; two-item nodes order their pair with one comparison (:270-281,
// an unsorted swap: equal keys DO swap), one-item nodes hold the item twice. The
// tree's shape depends on n alone and the axes on the seed alone, so nothing about
// the schedule is data-dependent and the device derives it on the fly:
//
//   the shape    a position's node at depth L is found by descending from the root
//                through the n / 2 splits (left child = the first count / 2 items);
//                its preorder index adds 1 per step plus, on a right step, the size
//                of the skipped left subtree, size(c) = 2 leaves(c) - 1 with
//                leaves(c) = 2^(k-1) + min(c - 2^k, 2^(k-1)) for c in (2^k, 2^(k+1)]
//                (the pieces of <= 2 items recursive halving leaves; 1 for c <= 2)
//   the axes     node k in preorder takes the k-th accepted draw of the split-axis
//                stream (AxisStream in lower.cpp: Philox4x32-10, key = seed, block b
//                = counter (b, 0, 0, 0); rand's gen_range(0..=2) rejects a word when
//                the low half of word * 3 exceeds 3 * 2^30 - 1): draw flags, one
//                exclusive scan, a scatter of the accepted axes
//   level_keys   composite 64-bit key per position: (start of its node << 32) |
//                total-order bits of key[axis] for nodes of > 2 items; positions in
//                finished leaves get (position << 32), which keeps them in place
//   radix sort   rocPRIM radix_sort_pairs over (key, item) — stable, so equal keys
//                keep the order the parent's sort left, as the stable merge sort does
//   deep_levels  from the first depth whose nodes hold at most kDeepMax items, one
//                workgroup finishes each node's subtree: its items stay in registers
//                and LDS, each remaining depth one stable block radix sort of the
//                same composite key over the node's own range
//   pair_order   the two-item leaves' single comparison, applied once at the end
//                (leaves are never touched by a deeper level)
//
// The host recursion does the same n log n work per level in a single thread.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

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

// Pieces of <= 2 items the recursive halving of c items leaves, and the nodes of that subtree.
__host__ __device__ inline uint32_t leaves_of(uint32_t c) {
    if (c <= 2u) return 1u;
    const uint32_t k = 31u - (uint32_t)__builtin_clz(c - 1u);  // c in (2^k, 2^(k+1)]
    const uint32_t half = 1u << (k - 1u), over = c - (1u << k);
    return half + (over < half ? over : half);
}
__host__ __device__ inline uint32_t nodes_of(uint32_t c) { return 2u * leaves_of(c) - 1u; }

// The node at depth L that holds position i (of the subtree (s, c) at preorder index pre
// and depth L0 <= L): its start, count and preorder index; `leaf` when a node of <= 2
// items above depth L holds i (it is never split further).
struct NodeAt {
    uint32_t s, c, pre;
    bool leaf;
};
__device__ inline NodeAt node_at(uint32_t i, uint32_t s, uint32_t c, uint32_t pre, uint32_t L0, uint32_t L) {
    for (uint32_t d = L0; d < L; ++d) {
        if (c <= 2u) return {s, c, pre, true};
        const uint32_t mid = c / 2u;
        if (i < s + mid) {
            pre += 1u;
            c = mid;
        } else {
            pre += 1u + nodes_of(mid);
            s += mid;
            c -= mid;
        }
    }
    return {s, c, pre, c <= 2u};
}

// f32 total_cmp order as an unsigned key (see above) of item `item`'s key on node `pre`'s axis.
__device__ inline uint32_t node_key(const float* __restrict__ keys, const uint8_t* __restrict__ axis, uint32_t pre,
                                    uint32_t item) {
    return total_order_bits(keys[3u * item + axis[pre]]);
}

// The split-axis stream: word w of Philox block b = w / 4 (counter (b, 0, 0, 0), key = seed);
// flag[w] = 1 when gen_range(0..=2) accepts it.
__device__ inline uint32_t mulhi_lo(uint32_t a, uint32_t b, uint32_t* lo) {
    const uint64_t p = (uint64_t)a * b;
    *lo = (uint32_t)p;
    return (uint32_t)(p >> 32);
}
__device__ inline uint4 philox_block(uint32_t c0, uint32_t k0, uint32_t k1) {
    uint32_t c1 = 0u, c2 = 0u, c3 = 0u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t lo0, lo1;
        const uint32_t hi0 = mulhi_lo(0xD2511F53u, c0, &lo0), hi1 = mulhi_lo(0xCD9E8D57u, c2, &lo1);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}
constexpr uint32_t kAxisZone = (3u << 30) - 1u;
__global__ __launch_bounds__(256) void axis_draws(uint32_t k0, uint32_t k1, uint32_t nblocks, uint32_t* __restrict__ flag,
                                                  uint8_t* __restrict__ val) {
    for (uint32_t b = blockIdx.x * 256u + threadIdx.x; b < nblocks; b += gridDim.x * 256u) {
        const uint4 w = philox_block(b, k0, k1);
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t lo;
            const uint32_t hi = mulhi_lo(ws[j], 3u, &lo);
            flag[4u * b + j] = lo <= kAxisZone ? 1u : 0u;
            val[4u * b + j] = (uint8_t)hi;
        }
    }
}
__global__ __launch_bounds__(256) void axis_scatter(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos,
                                                    const uint8_t* __restrict__ val, uint32_t nwords, uint32_t nnodes,
                                                    uint8_t* __restrict__ axis) {
    for (uint32_t w = blockIdx.x * 256u + threadIdx.x; w < nwords; w += gridDim.x * 256u)
        if (flag[w] && pos[w] < nnodes) axis[pos[w]] = val[w];
}

// One depth L of the global phase: the composite key of every position.
__global__ __launch_bounds__(256) void level_keys(const float* __restrict__ keys, const uint32_t* __restrict__ order,
                                                  const uint8_t* __restrict__ axis, uint32_t L, uint32_t n,
                                                  uint64_t* __restrict__ out) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const NodeAt a = node_at(i, 0u, n, 0u, 0u, L);
        out[i] = a.leaf ? (uint64_t)i << 32 : ((uint64_t)a.s << 32) | node_key(keys, axis, a.pre, order[i]);
    }
}

// Depths [L0, L1) of the subtree of the depth-L0 node with path bits blockIdx.x (count <=
// kDeepMax), in place on its range of `order`.
constexpr uint32_t kDeepThreads = 256u, kDeepItems = 8u, kDeepMax = kDeepThreads * kDeepItems;
__global__ __launch_bounds__(256) void deep_levels(const float* __restrict__ keys, uint32_t* __restrict__ order,
                                                   const uint8_t* __restrict__ axis, uint32_t n, uint32_t L0, uint32_t L1) {
    using Sort = rocprim::block_radix_sort<uint64_t, kDeepThreads, kDeepItems, uint32_t>;
    __shared__ typename Sort::storage_type storage;
    uint32_t s0 = 0u, c0 = n, pre0 = 0u;  // the subtree root: follow the path bits, most significant first
    for (uint32_t d = 0; d < L0; ++d) {
        const uint32_t mid = c0 / 2u;
        if ((blockIdx.x >> (L0 - 1u - d)) & 1u) {
            pre0 += 1u + nodes_of(mid);
            s0 += mid;
            c0 -= mid;
        } else {
            pre0 += 1u;
            c0 = mid;
        }
    }
    uint32_t item[kDeepItems];
    uint64_t key[kDeepItems];
#pragma unroll
    for (uint32_t i = 0; i < kDeepItems; ++i) {
        const uint32_t p = threadIdx.x * kDeepItems + i;  // blocked: the sort's own arrangement
        item[i] = p < c0 ? order[s0 + p] : 0u;
    }
    for (uint32_t L = L0; L < L1; ++L) {
#pragma unroll
        for (uint32_t i = 0; i < kDeepItems; ++i) {
            const uint32_t p = threadIdx.x * kDeepItems + i;
            if (p >= c0) {
                key[i] = ~0ull;  // padding sorts last (and after the items: the sort is stable)
                continue;
            }
            const NodeAt a = node_at(p, 0u, c0, pre0, L0, L);
            key[i] = a.leaf ? (uint64_t)p << 32 : ((uint64_t)a.s << 32) | node_key(keys, axis, a.pre, item[i]);
        }
        Sort().sort(key, item, storage, 0u, 32u + 11u);  // local starts < kDeepMax = 2^11
        __syncthreads();
    }
#pragma unroll
    for (uint32_t i = 0; i < kDeepItems; ++i) {
        const uint32_t p = threadIdx.x * kDeepItems + i;
        if (p < c0) order[s0 + p] = item[i];
    }
}

__global__ void iota(uint32_t* __restrict__ order, uint32_t n) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) order[i] = i;
}

// bvh.rs:270-281: (objects[0], objects[1]) if compare(0, 1) == Less, else swapped; one
// thread per position, acting at the first position of each two-item leaf.
__global__ void pair_order(const float* __restrict__ keys, uint32_t* __restrict__ order,
                           const uint8_t* __restrict__ axis, uint32_t n) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const NodeAt a = node_at(i, 0u, n, 0u, 0u, 64u);
        if (a.c != 2u || a.s != i) continue;
        const uint32_t x = order[i], y = order[i + 1u];
        if (!(node_key(keys, axis, a.pre, x) < node_key(keys, axis, a.pre, y))) {
            order[i] = y;
            order[i + 1u] = x;
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
    const uint32_t nnodes = nodes_of(n);
    // Depth L holds nodes of at most ceil(n / 2^L) items: sorting ends at the first depth where
    // that is <= 2 (Lend); the workgroup phase starts at the first depth where it is <= kDeepMax.
    auto maxc = [n](uint32_t L) { return L >= 32u ? 1u : (uint32_t)(((uint64_t)n + (1ull << L) - 1u) >> L); };
    uint32_t Lend = 0, L0 = 0;
    while (maxc(Lend) > 2u) ++Lend;
    while (L0 < Lend && maxc(L0) > kDeepMax) ++L0;
    DevBufs b;
    uint32_t *alt = nullptr, *flag = nullptr, *pos = nullptr;
    uint8_t *val = nullptr, *axis = nullptr;
    uint64_t *k0 = nullptr, *k1 = nullptr;
    hipError_t e;
    if ((e = b.alloc(&alt, n)) || (e = b.alloc(&k0, n)) || (e = b.alloc(&k1, n)) || (e = b.alloc(&axis, nnodes)))
        return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc (BVH build): ") + hipGetErrorString(e));
    (void)hipGetLastError();
    // The split axes of all nodes in preorder: about 4/3 draws per node; a shortfall (never seen
    // at these sizes) doubles the words drawn.
    const uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
    for (uint64_t words = ((uint64_t)nnodes * 3u / 2u + 1024u + 3u) & ~3ull;; words *= 2u) {
        if (words > 0xFFFFFFF0ull) return rthost::set_error(RT_ERR_UNSUPPORTED, "BVH too large for the axis stream");
        const uint32_t nw = (uint32_t)words;
        DevBufs w;
        size_t scan_bytes = 0;
        uint8_t* scan_tmp = nullptr;
        if ((e = w.alloc(&flag, nw)) || (e = w.alloc(&pos, nw)) || (e = w.alloc(&val, nw)))
            return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc (axis stream): ") + hipGetErrorString(e));
        if ((e = rocprim::exclusive_scan(nullptr, scan_bytes, flag, pos, 0u, (size_t)nw, rocprim::plus<uint32_t>(), st)) ||
            (e = w.alloc(&scan_tmp, scan_bytes)))
            return rthost::set_error(RT_ERR_HIP, std::string("axis scan setup: ") + hipGetErrorString(e));
        hipLaunchKernelGGL(axis_draws, dim3(grid_for(nw / 4u)), dim3(256), 0, st, key0, key1, nw / 4u, flag, val);
        if ((e = rocprim::exclusive_scan(scan_tmp, scan_bytes, flag, pos, 0u, (size_t)nw, rocprim::plus<uint32_t>(), st)))
            return rthost::set_error(RT_ERR_HIP, std::string("axis scan: ") + hipGetErrorString(e));
        uint32_t last[2] = {0u, 0u};
        if ((e = hipMemcpyAsync(&last[0], pos + nw - 1u, 4u, hipMemcpyDeviceToHost, st)) ||
            (e = hipMemcpyAsync(&last[1], flag + nw - 1u, 4u, hipMemcpyDeviceToHost, st)) ||
            (e = hipStreamSynchronize(st)))
            return rthost::set_error(RT_ERR_HIP, std::string("axis count: ") + hipGetErrorString(e));
        if ((uint64_t)last[0] + last[1] < nnodes) continue;
        hipLaunchKernelGGL(axis_scatter, dim3(grid_for(nw)), dim3(256), 0, st, flag, pos, val, nw, nnodes, axis);
        if ((e = hipStreamSynchronize(st)))  // the scratch buffers are freed at the end of this scope
            return rthost::set_error(RT_ERR_HIP, std::string("axis scatter: ") + hipGetErrorString(e));
        break;
    }
    const uint32_t end_bit = 32u + bits_for(n - 1u);
    size_t tmp_bytes = 0;
    if ((e = rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, d_order, alt, (size_t)n, 0u, end_bit, st)))
        return rthost::set_error(RT_ERR_HIP, std::string("radix sort query: ") + hipGetErrorString(e));
    uint8_t* tmp = nullptr;
    if ((e = b.alloc(&tmp, tmp_bytes)))
        return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc (sort scratch): ") + hipGetErrorString(e));
    uint32_t* cur = d_order;
    uint32_t* nxt = alt;
    hipLaunchKernelGGL(iota, dim3(grid_for(n)), dim3(256), 0, st, cur, n);
    for (uint32_t L = 0; L < L0; ++L) {
        hipLaunchKernelGGL(level_keys, dim3(grid_for(n)), dim3(256), 0, st, d_keys, cur, axis, L, n, k0);
        if ((e = rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, cur, nxt, (size_t)n, 0u, end_bit, st)))
            return rthost::set_error(RT_ERR_HIP, std::string("radix sort: ") + hipGetErrorString(e));
        std::swap(cur, nxt);
    }
    if (L0 < Lend)  // every depth-L0 node exists: the depths above hold > kDeepMax >= 3 items per node
        hipLaunchKernelGGL(deep_levels, dim3(1u << L0), dim3(kDeepThreads), 0, st, d_keys, cur, axis, n, L0, Lend);
    hipLaunchKernelGGL(pair_order, dim3(grid_for(n)), dim3(256), 0, st, d_keys, cur, axis, n);
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
