// gather.hip — frame assembly for one process per GPU.
//
// The reference composites its tiles into one image on the host
// (src/renderer.rs:63-95). Here rank r of n renders the 8x8 blocks b with
// b % n == r (rt_render_params.shard_index / shard_count, the block interleave
// the trace kernel uses) into a full-frame device image; rt_shard_pack moves
// those blocks into a dense buffer (64 pixel slots per block, blocks in order),
// the rank copies it with one hipMemcpyAsync into its slot of a buffer shared
// with rank 0, and rank 0 scatters all n shards back with rt_shard_unpack.
// Pure copies: the assembled image is the one-device image bit for bit. Both
// kernels are HBM-bound (12 B read + 12 B written per pixel).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string.h>

#include <map>
#include <mutex>
#include <string>

#include "../../include/rt.h"
#include "common.hpp"

namespace {

struct Grid {
    uint32_t bx, nb;  // blocks per row, blocks in the frame
};
Grid grid_of(uint32_t w, uint32_t h) { return Grid{(w + 7u) / 8u, ((w + 7u) / 8u) * ((h + 7u) / 8u)}; }

// blocks of rank r: b = r, r + n, ... < nb
__host__ __device__ inline uint64_t blocks_of(uint32_t nb, uint32_t r, uint32_t n) {
    return r < nb ? (uint64_t)(nb - r + n - 1u) / n : 0u;
}
// blocks of ranks 0..r-1: r * floor(nb / n) + min(r, nb % n)
__host__ __device__ inline uint64_t blocks_before(uint32_t nb, uint32_t r, uint32_t n) {
    const uint32_t q = nb / n, m = nb % n;
    return (uint64_t)r * q + (r < m ? r : m);
}

// thread = (k-th block of the rank, pixel slot p): packed[(k * 64 + p) * 3 + c]
__global__ __launch_bounds__(256) void shard_pack(const float* __restrict__ img, uint32_t w, uint32_t h, uint32_t bx,
                                                  uint32_t r, uint32_t n, uint64_t slots, float* __restrict__ packed) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * 256u) {
        const uint64_t k = i >> 6;
        const uint32_t p = (uint32_t)(i & 63u);
        const uint64_t b = r + k * n;
        const uint32_t x = (uint32_t)(b % bx) * 8u + (p & 7u), y = (uint32_t)(b / bx) * 8u + (p >> 3);
        if (x >= w || y >= h) continue;
        const float* src = img + ((uint64_t)y * w + x) * 3u;
        float* dst = packed + i * 3u;
        dst[0] = src[0];
        dst[1] = src[1];
        dst[2] = src[2];
    }
    // System-scope release: this thread's stores are written back past the L2 before it ends,
    // so a peer that reads the packed shard over xGMI after the host has seen this stream
    // complete (rt_shard_pull_unpack) finds them in memory whatever release scope the
    // runtime gives the dispatch's end.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// Pull form of the gather: rank 0 scatters the blocks of ranks 1..n-1 straight from their
// packed-shard buffers (peer memory mapped with rt_ipc_open, read over xGMI) into its image;
// its own blocks are already there. thread = (frame block b with b % n != 0, pixel slot p).
constexpr uint32_t kMaxPullRanks = 64;
struct PeerShards {
    const float* p[kMaxPullRanks];  // p[r]: rank r's packed shard (k-th block of the rank at k * 64 slots)
};
__global__ __launch_bounds__(256) void shard_pull_unpack(PeerShards peers, uint32_t w, uint32_t h, uint32_t bx,
                                                         uint32_t nb, uint32_t n, float* __restrict__ img) {
    // System-scope acquire: the L1 / L2 lines a previous step left are invalidated before any
    // peer word is read (with the writer's release in shard_pack and the host barrier between
    // the writer's stream completion and this launch, the LLVM AMDGPU memory model makes every
    // packed word visible here), and each peer word is read with a system-scope load.
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint64_t slots = (uint64_t)nb * 64u;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * 256u) {
        const uint32_t b = (uint32_t)(i >> 6), p = (uint32_t)(i & 63u);
        const uint32_t r = b % n;
        if (r == 0u) continue;
        const uint32_t x = (b % bx) * 8u + (p & 7u), y = (b / bx) * 8u + (p >> 3);
        if (x >= w || y >= h) continue;
        const float* src = peers.p[r] + ((uint64_t)(b / n) * 64u + p) * 3u;
        float* dst = img + ((uint64_t)y * w + x) * 3u;
#pragma unroll
        for (int c = 0; c < 3; ++c)
            dst[c] = __hip_atomic_load(src + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// thread = (frame block b, pixel slot p); shard b % n holds it at slot b / n
__global__ __launch_bounds__(256) void shard_unpack(const float* __restrict__ packed, uint32_t w, uint32_t h,
                                                    uint32_t bx, uint32_t nb, uint32_t n, float* __restrict__ img) {
    const uint64_t slots = (uint64_t)nb * 64u;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * 256u) {
        const uint32_t b = (uint32_t)(i >> 6), p = (uint32_t)(i & 63u);
        const uint32_t x = (b % bx) * 8u + (p & 7u), y = (b / bx) * 8u + (p >> 3);
        if (x >= w || y >= h) continue;
        const uint32_t r = b % n;
        const uint64_t slot = (blocks_before(nb, r, n) + b / n) * 64u + p;
        const float* src = packed + slot * 3u;
        float* dst = img + ((uint64_t)y * w + x) * 3u;
        dst[0] = src[0];
        dst[1] = src[1];
        dst[2] = src[2];
    }
}

uint32_t launch_blocks(uint64_t work) {
    const uint64_t b = (work + 255u) / 256u;
    return (uint32_t)(b < 8192u ? (b ? b : 1u) : 8192u);
}

int hip_fail(hipError_t e, const char* what) {
    return rthost::set_error(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

extern "C" {

uint64_t rt_shard_floats(uint32_t width, uint32_t height, uint32_t rank, uint32_t n) {
    if (n == 0) return 0;
    return blocks_of(grid_of(width, height).nb, rank, n) * 64u * 3u;
}

uint64_t rt_shard_offset(uint32_t width, uint32_t height, uint32_t rank, uint32_t n) {
    if (n == 0) return 0;
    const uint32_t r = rank < n ? rank : n;
    return blocks_before(grid_of(width, height).nb, r, n) * 64u * 3u;
}

int rt_shard_pack(const float* d_image, uint32_t width, uint32_t height, uint32_t rank, uint32_t n, float* d_packed,
                  void* stream) {
    rthost::clear_error();
    if (n == 0 || rank >= n || width == 0 || height == 0)
        return rthost::set_error(RT_ERR_INVALID, "rt_shard_pack: empty image or rank >= n");
    const Grid g = grid_of(width, height);
    const uint64_t slots = blocks_of(g.nb, rank, n) * 64u;
    if (slots == 0) return RT_OK;  // a rank without blocks (n > blocks) ships nothing
    if (!d_image || !d_packed) return rthost::set_error(RT_ERR_INVALID, "rt_shard_pack: NULL buffer");
    (void)hipGetLastError();
    hipLaunchKernelGGL(shard_pack, dim3(launch_blocks(slots)), dim3(256), 0, (hipStream_t)stream, d_image, width,
                       height, g.bx, rank, n, slots, d_packed);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RT_OK : hip_fail(e, "shard_pack launch");
}

int rt_shard_unpack(const float* d_packed_all, uint32_t width, uint32_t height, uint32_t n, float* d_image,
                    void* stream) {
    rthost::clear_error();
    if (!d_packed_all || !d_image || n == 0 || width == 0 || height == 0)
        return rthost::set_error(RT_ERR_INVALID, "rt_shard_unpack: NULL buffer, empty image or n == 0");
    const Grid g = grid_of(width, height);
    (void)hipGetLastError();
    hipLaunchKernelGGL(shard_unpack, dim3(launch_blocks((uint64_t)g.nb * 64u)), dim3(256), 0, (hipStream_t)stream,
                       d_packed_all, width, height, g.bx, g.nb, n, d_image);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RT_OK : hip_fail(e, "shard_unpack launch");
}

int rt_shard_pull_unpack(const float* const* d_peer_packed, uint32_t width, uint32_t height, uint32_t n,
                         float* d_image, void* stream) {
    rthost::clear_error();
    if (!d_peer_packed || !d_image || n == 0 || width == 0 || height == 0)
        return rthost::set_error(RT_ERR_INVALID, "rt_shard_pull_unpack: NULL buffer, empty image or n == 0");
    if (n > kMaxPullRanks) return rthost::set_error(RT_ERR_INVALID, "rt_shard_pull_unpack: more than 64 ranks");
    if (n == 1) return RT_OK;
    const Grid g = grid_of(width, height);
    PeerShards peers{};
    for (uint32_t r = 1; r < n; ++r) {
        if (blocks_of(g.nb, r, n) && !d_peer_packed[r])
            return rthost::set_error(RT_ERR_INVALID, "rt_shard_pull_unpack: NULL peer buffer");
        peers.p[r] = d_peer_packed[r];
    }
    (void)hipGetLastError();
    hipLaunchKernelGGL(shard_pull_unpack, dim3(launch_blocks((uint64_t)g.nb * 64u)), dim3(256), 0,
                       (hipStream_t)stream, peers, width, height, g.bx, g.nb, n, d_image);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? RT_OK : hip_fail(e, "shard_pull_unpack launch");
}

// Peer transport (frame_gather.FrameGather's "ipc" path): rank 0 exports its gather
// buffer with hipIpcGetMemHandle, every other rank maps it (hipIpcOpenMemHandle) and copies
// its packed shard straight into its slot, device to device over xGMI, one hop instead of
// the D2H + H2D bounce through host memory. The buffer may sit inside a larger allocation
// (a caching allocator's segment): the handle names the allocation's base and the offset
// travels in the last 8 bytes of the RT_IPC_HANDLE_BYTES record.
struct IpcRecord {
    hipIpcMemHandle_t h;
    uint64_t offset;
};
static_assert(sizeof(IpcRecord) <= RT_IPC_HANDLE_BYTES, "IPC record size");
namespace {
std::mutex g_ipc_mu;
std::map<uintptr_t, void*> g_ipc_base;  // mapped pointer handed out -> base hipIpcOpenMemHandle returned
struct DevSwitch {
    int prev = -1;
    hipError_t e;
    explicit DevSwitch(int d) {
        (void)hipGetDevice(&prev);
        e = hipSetDevice(d);
    }
    ~DevSwitch() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
}  // namespace

int rt_ipc_export(const void* d_ptr, int device, uint8_t handle[RT_IPC_HANDLE_BYTES]) {
    rthost::clear_error();
    if (!d_ptr || !handle) return rthost::set_error(RT_ERR_INVALID, "rt_ipc_export: NULL argument");
    DevSwitch ds(device);
    if (ds.e != hipSuccess) return hip_fail(ds.e, "hipSetDevice");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d_ptr);
    if (e != hipSuccess) return hip_fail(e, "hipMemGetAddressRange");
    IpcRecord rec{};
    if ((e = hipIpcGetMemHandle(&rec.h, (void*)base)) != hipSuccess) return hip_fail(e, "hipIpcGetMemHandle");
    rec.offset = (uint64_t)((const char*)d_ptr - (const char*)base);
    memset(handle, 0, RT_IPC_HANDLE_BYTES);
    memcpy(handle, &rec, sizeof rec);
    return RT_OK;
}

int rt_ipc_open(const uint8_t handle[RT_IPC_HANDLE_BYTES], int device, void** d_ptr) {
    rthost::clear_error();
    if (!handle || !d_ptr) return rthost::set_error(RT_ERR_INVALID, "rt_ipc_open: NULL argument");
    *d_ptr = nullptr;
    IpcRecord rec;
    memcpy(&rec, handle, sizeof rec);
    DevSwitch ds(device);
    if (ds.e != hipSuccess) return hip_fail(ds.e, "hipSetDevice");
    void* base = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&base, rec.h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return hip_fail(e, "hipIpcOpenMemHandle");
    void* p = (char*)base + rec.offset;
    {
        std::lock_guard<std::mutex> lk(g_ipc_mu);
        g_ipc_base[(uintptr_t)p] = base;
    }
    *d_ptr = p;
    return RT_OK;
}

int rt_ipc_close(void* d_ptr, int device) {
    rthost::clear_error();
    if (!d_ptr) return RT_OK;
    void* base = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_ipc_mu);
        auto it = g_ipc_base.find((uintptr_t)d_ptr);
        if (it == g_ipc_base.end()) return rthost::set_error(RT_ERR_INVALID, "rt_ipc_close: pointer not from rt_ipc_open");
        base = it->second;
        g_ipc_base.erase(it);
    }
    DevSwitch ds(device);
    if (ds.e != hipSuccess) return hip_fail(ds.e, "hipSetDevice");
    hipError_t e = hipIpcCloseMemHandle(base);
    return e == hipSuccess ? RT_OK : hip_fail(e, "hipIpcCloseMemHandle");
}

int rt_copy_async(void* d_dst, const void* d_src, uint64_t bytes, void* stream) {
    rthost::clear_error();
    if (bytes == 0) return RT_OK;
    if (!d_dst || !d_src) return rthost::set_error(RT_ERR_INVALID, "rt_copy_async: NULL buffer");
    hipError_t e = hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    return e == hipSuccess ? RT_OK : hip_fail(e, "hipMemcpyAsync (shard to rank 0)");
}

}  // extern "C"
