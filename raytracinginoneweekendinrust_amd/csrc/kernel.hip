// kernel.hip — the MI355X (gfx950 / CDNA4) path-tracing hot path.
//
// One 64-lane wave renders one 8x8 pixel block; lane = pixel. Each lane walks
// its pixel's samples in order (src/renderer.rs:140-147) with PATH
// REGENERATION: a lane whose path ends accumulates and immediately starts its
// next camera sample, so every loop trip is one ray segment for every live
// lane and no lane idles while a neighbour finishes a long path.
//
// Per segment (src/ray.rs:32-62): the top-level HittableList is walked in
// order with a wave-uniform loop (entries are read with scalar loads), each
// entry applies its Translate/RotateY chain, then tests a primitive, a cube, a
// BVH (per-lane DFS stack in LDS, lane-strided so pushes never bank-conflict)
// or a ConstantMedium. Only (t, entry, primitive) is kept per candidate; the
// HitRecord of the winning candidate is rebuilt once, with the same arithmetic
// the candidate test used, before Material::scatter / emit.
//
// Bit-exactness with the CPU oracle: built with -ffp-contract=off, correctly
// rounded f32/f64 division and square root, rt_numeric_spec.h transcendentals,
// and the reference's operation order (glam 0.22) everywhere. No MFMA: the path
// has no dense contraction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "../../include/rt_numeric_spec.h"
#include "common.hpp"
#include "device_scene.hpp"
#include "lower.hpp"

using rtdev::DevCamera;
using rtdev::DevEntry;
using rtdev::DevMaterial;
using rtdev::DevParams;
using rtdev::DevScene;
using rtdev::DevTexture;
using rtdev::f4;

#define RT_DEV __device__ __forceinline__

namespace {

constexpr float kInf = __builtin_inff();

// ---------------------------------------------------------------------------
// Region profiler (diagnostic build only: -DRT_PROFILE_REGIONS -> librtamd_prof.so,
// see tools/region_profile.py). Per region: wave cycles (s_memtime), wave
// executions and active lanes at region end; accumulated per wave in LDS by the
// first active lane, flushed to g_prof once per wave. Compiles to nothing in the
// product library.
// ---------------------------------------------------------------------------
enum ProfRegion : uint32_t {
    kPrRefill = 0, kPrSegment, kPrWorld, kPrRecord, kPrEmit, kPrScatter, kPrMarble, kPrStore,
    kPrChecker, kPrImage, kPrUnitSphere, kPrDielectric, kPrLambert, kPrMetal, kPrIso, kPrLog,
    kPrEntry0 = 16, kPrEntryLast = 43, kPrBvhTrip = 44, kPrLeafTest = 45, kPrBvhSetup = 46, kPrBvhPush = 47,
    kPrBvhPop = 48, kPrBvhCall = 49, kPrCount = 52
};
// traversal mode bits (bvh_hit): kModeExact = RT_FLAG_EXACT_BVH; the rest come
// from DevParams::tune (rt_set_option(RT_OPT_TUNE), diagnostics / A-B runs).
constexpr uint32_t kModeExact = 1u, kModeNoLeafBoxes = 2u, kModeNoPermLds = 32u, kModeW3 = 64u,
                   kModeNoPretest = 128u, kModeReplayRef = 1u << 16;  // ReplayRef: the replay pass runs trace_samples<1>
// NoStream: no streaming replay pass beside the fast kernel (the serialized pass takes every
// handed-over sample after it); the tests cover both
constexpr uint32_t kModeNoStream = 1u << 17;
// EXPERIMENT ONLY (RT_OPT_TUNE, not exact): closest-hit pruning also on BVHs the proof does not
// cover (triangles, moving spheres), to measure what an exact bound for them could gain. Compiled
// into the audit and ablation builds only: the product library rejects the bit (kTuneAccepted).
constexpr uint32_t kModePruneAllExp = 1u << 20;
#if defined(RT_LEAF_AUDIT) || defined(RT_ABLATE)
constexpr bool kPruneAllExpBuild = true;
#else
constexpr bool kPruneAllExpBuild = false;
#endif
// Block order: a shard's blocks are taken last block first (bottom image rows first), so the
// upper rows, which in every BASELINE framing hold the background and end their paths after a
// segment or two, are the work left when the pool runs dry and the drain is short (one rank of
// 8: C3 69.7 -> 68.0 ms, C1 -3%). BlocksForward (RT_OPT_TUNE, A/B only) restores
// the top-first order. Either order gives the same bits (samples are keyed by pixel and index).
constexpr uint32_t kModeBlocksForward = 1u << 21;
// W4 (RT_OPT_TUNE, A/B only): the 4-wave instance also for the presets that prefer 3 (below).
constexpr uint32_t kModeW4 = 1u << 22;
// MbShrink (RT_OPT_TUNE, audit build only): halves the medium-first estimate (world_hit)
[[maybe_unused]] constexpr uint32_t kModeMbShrink = 1u << 29;
// The RT_OPT_TUNE bits a build honours. Every bit of the product library leaves the image bits
// unchanged (instance choice, block order, replay-pass form, leaf postponement's q in bits 24-27,
// switching exact shortcuts off); rt_set_option refuses any other bit with RT_ERR_INVALID, so no
// caller can leave parity through the C ABI (the boundary contract: renderer.rs:42-52 has no knob
// that changes results). The audit, ablation and A/B builds add their diagnostic bits.
constexpr uint32_t kTuneExact = kModeNoLeafBoxes | kModeNoPermLds | kModeW3 | kModeNoPretest | kModeReplayRef |
                                kModeNoStream | kModeBlocksForward | kModeW4 | (15u << 24);
constexpr uint32_t kTuneAccepted = kTuneExact
#if defined(RT_LEAF_AUDIT) || defined(RT_ABLATE)
                                   | kModePruneAllExp
#endif
#ifdef RT_LEAF_AUDIT
                                   | kModeMbShrink
#endif
#ifdef RT_ABLATE
                                   | (31u << 8)  // kAb* below
#endif
#ifdef RT_EXP_STRIDE
                                   | (1u << 23)
#endif
    ;
#ifdef RT_ABLATE
// Ablation build (librtamd_ablate.so, diagnostics only): RT_OPT_TUNE bits that run a
// piece of work twice (results of the copy discarded through an opaque test),
// so the time delta prices that work without changing any path.
constexpr uint32_t kAbLeaf2 = 1u << 8, kAbKeys2 = 1u << 9, kAbBvh2 = 1u << 10, kAbMedium2 = 1u << 11,
                   kAbGeom2 = 1u << 12;
#define ABLATE(bit, ...) do { if (mode & (bit)) { __VA_ARGS__ } } while (0)
#else
#define ABLATE(bit, ...) do { } while (0)
#endif
#ifdef RT_PROFILE_REGIONS
constexpr uint32_t kProfCopies = 64;  // flush targets spread over blockIdx to keep atomics uncontended
constexpr uint32_t kProfWords = 3 * kPrCount + 16;  // region triples, then the two visit histograms
__device__ unsigned long long g_prof[kProfCopies * kProfWords];
// per-wave start / end clock (s_memrealtime, 100 MHz) of the fast kernel's last launch: the
// ramp at the start and the drain at the end of a launch (tools/region_profile.py --waves)
constexpr uint32_t kProfWaves = 8192;
__device__ unsigned long long g_wave_t[2 * kProfWaves];
// segments executed per 200 us since each wave's start (the fast kernel's throughput over a launch)
constexpr uint32_t kTpBuckets = 4096, kTpTicks = 20000u;  // s_memrealtime ticks (100 MHz) per bucket
__device__ unsigned long long g_tp_hist[kTpBuckets];
// streaming replay pass events: (s_memrealtime, claimed entry or ~0 at the wave's exit)
constexpr uint32_t kRoleEvents = 4096;
__device__ unsigned long long g_role_ev[2 * kRoleEvents];
__device__ unsigned g_role_n;
// block-row band [g_prof_rows[0], g_prof_rows[1]) the profiling build renders (rt_prof_rows): the
// launch's pool holds only that band's blocks (rt_render_launch_camera offsets the block map)
uint32_t g_prof_rows[2] = {0u, 0xffffffffu};
__device__ __forceinline__ void role_event(uint32_t what) {
    const unsigned i = atomicAdd(&g_role_n, 1u);
    if (i < kRoleEvents) {
        g_role_ev[2u * i] = __builtin_amdgcn_s_memrealtime();
        g_role_ev[2u * i + 1u] = what;
    }
}
__shared__ unsigned long long prof_lds[kProfWords];
// per-traversal node-visit histograms (prof_lds[3 * kPrCount + bin]: lanes,
// [3 * kPrCount + 8 + bin]: the wave's max per call); bins 0,1,2,3-4,5-8,9-16,17-32,33+
__device__ __forceinline__ uint32_t trips_bin(uint32_t n) {
    return n == 0u ? 0u : n == 1u ? 1u : n == 2u ? 2u : n <= 4u ? 3u : n <= 8u ? 4u : n <= 16u ? 5u : n <= 32u ? 6u : 7u;
}
__device__ __forceinline__ void prof_init() {
    for (uint32_t i = threadIdx.x; i < kProfWords; i += blockDim.x) prof_lds[i] = 0u;
}
__device__ __forceinline__ void prof_flush() {
    unsigned long long* dst = g_prof + (blockIdx.x % kProfCopies) * kProfWords;
    for (uint32_t i = threadIdx.x; i < kProfWords; i += blockDim.x)
        if (prof_lds[i]) atomicAdd(&dst[i], prof_lds[i]);
}
#define PROF_T0(name) const uint64_t name = __builtin_amdgcn_s_memtime()
#define PROF_ADD(region, t0) prof_add((region), (t0))
__device__ __forceinline__ void prof_add(uint32_t region, uint64_t t0) {
    uint64_t dt = __builtin_amdgcn_s_memtime() - t0;
    uint64_t m = __ballot(1);
    if (__lane_id() == (uint32_t)__builtin_ctzll(m)) {
        prof_lds[region] += dt;
        prof_lds[kPrCount + region] += 1u;
        prof_lds[2 * kPrCount + region] += (uint64_t)__popcll(m);
    }
}
#define PROF_INIT() prof_init()
#define PROF_FLUSH() prof_flush()
#else
#define PROF_T0(name) do { } while (0)
#define PROF_ADD(region, t0) do { } while (0)
#define PROF_INIT() do { } while (0)
#define PROF_FLUSH() do { } while (0)
#endif
#ifdef RT_LEAF_AUDIT
// Leaf-box audit (audit build, -DRT_LEAF_AUDIT -> librtamd_audit.so): leaves
// rejected by the conservative leaf test are tested anyway; a rejected leaf that would have
// produced a candidate is recorded here and printed when the scene is freed.
struct LeafAudit {
    float o[3], d[3], tmin, closest, t, box[6], delta;
    uint32_t code, rank, best_rank;
};
constexpr uint32_t kAuditMax = 64;
__device__ unsigned g_audit_count;
__device__ LeafAudit g_audit[kAuditMax];
// and every fast traversal is replayed with bvh_hit_reference; disagreements land here
struct TravAudit {
    float o[3], d[3], tmin, tmax, fast_t, ref_t;
    uint32_t fast_code, ref_code, root;
};
__device__ unsigned g_trav_audit_count;
// and every visited / pushed BVH node index and stack position is bounds-checked: a
// violation (e.g. a non-finite slab value steering the traversal) is counted and the
// traversal stops instead of faulting
__device__ unsigned g_bounds_audit_count;
__device__ TravAudit g_trav_audit[kAuditMax];
#endif

// ---------------------------------------------------------------------------
// vector math, glam 0.22 evaluation order
// ---------------------------------------------------------------------------
struct V {
    float x, y, z;
};
#ifdef RT_DEBUG_PIXEL
// Diagnostic builds only: records of one (pixel, sample)'s path, read back after the render
// (the host prints them to stderr). Plain stores, so the instrumented kernel stays close to the
// product's code.
constexpr uint32_t kDbgMax = 256;
__device__ uint32_t g_dbg[8 * kDbgMax];
__device__ unsigned g_dbg_n;
#ifndef RT_DEBUG_TRACE
#define RT_DEBUG_TRACE 1
#endif
#ifdef RT_DEBUG_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
void dbg_put(uint32_t tag, uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e,
                                     uint32_t f, uint32_t h) {
    const unsigned i = atomicAdd(&g_dbg_n, 1u);
    if (i < kDbgMax) {
        uint32_t* o = g_dbg + 8u * i;
        o[0] = tag; o[1] = a; o[2] = b; o[3] = c; o[4] = d; o[5] = e; o[6] = f; o[7] = h;
    }
}
#endif
RT_DEV V mk(float x, float y, float z) { return V{x, y, z}; }
RT_DEV V operator+(V a, V b) { return V{a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_DEV V operator-(V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_DEV V operator*(V a, V b) { return V{a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_DEV V operator*(float s, V a) { return V{s * a.x, s * a.y, s * a.z}; }
RT_DEV V operator-(V a) { return V{-a.x, -a.y, -a.z}; }
RT_DEV V divs(V a, float s) { return V{a.x / s, a.y / s, a.z / s}; }
RT_DEV float dot(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
RT_DEV V cross(V a, V b) { return V{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
RT_DEV float length(V a) { return __builtin_sqrtf(dot(a, a)); }
RT_DEV V normalize(V a) {
    float r = 1.0f / length(a);
    return V{a.x * r, a.y * r, a.z * r};
}
RT_DEV float rs_min(float a, float b) {  // Rust f32::min (minnum)
    if (a != a) return b;
    if (b != b) return a;
    return a < b ? a : b;
}
RT_DEV float rs_clamp(float x, float lo, float hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
RT_DEV bool sign_negative(float x) { return (__float_as_uint(x) >> 31) != 0u; }
RT_DEV bool sign_negative_d(double x) { return (__double_as_longlong(x) >> 63) != 0; }
RT_DEV V xyz(f4 a) { return V{a.x, a.y, a.z}; }
// Scene rows are read through memcpy from their declared alignment, not by punning an f4
// pointer as float2 / float4 (no type-based aliasing assumption is involved in any load).
[[maybe_unused]] RT_DEV float2 ld2(const f4* p, uint32_t row) {  // the .xy half of row `row` (audit and ablation builds)
    float2 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p + row, 16), sizeof(v));
    return v;
}
RT_DEV f4 ld4(const f4* p) {
    f4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 16), sizeof(v));
    return v;
}
// Row loads at a 32-bit byte offset from a wave-uniform base (BVH4 nodes: 16-byte rows; the
// .xy halves of leaf rows at 8-byte granularity; single lanes of leaf rows).
RT_DEV f4 ld4_at(const f4* base, uint32_t byte_off) {
    f4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(reinterpret_cast<const char*>(base) + byte_off, 16), sizeof(v));
    return v;
}
RT_DEV float ld1_at(const f4* base, uint32_t byte_off) {
    float v;
    __builtin_memcpy(&v, __builtin_assume_aligned(reinterpret_cast<const char*>(base) + byte_off, 4), sizeof(v));
    return v;
}
RT_DEV float2 ld2_at(const f4* base, uint32_t byte_off) {
    float2 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(reinterpret_cast<const char*>(base) + byte_off, 8), sizeof(v));
    return v;
}
// Wave-uniform reads of the read-only scene records (top-level entries, their transforms, run and
// boundary records) through the constant address space: at a uniform address the backend loads
// them with s_load into SGPRs through the scalar cache, where a global load waits on the vector
// memory path (two dependent trips per entry: the walls of C4 and C5 took 2,600 wave cycles each).
#ifndef RT_SCALAR_ENTRIES
#define RT_SCALAR_ENTRIES 1
#endif
#if RT_SCALAR_ENTRIES
#define RT_AS4 __attribute__((address_space(4)))
#else
#define RT_AS4
#endif
template <class T>
RT_DEV const RT_AS4 T* cst(const T* p) {
    return (const RT_AS4 T*)p;
}
RT_DEV f4 ld4c(const f4* p) {
    const RT_AS4 f4* q = cst(p);
    return f4{q->x, q->y, q->z, q->w};
}

struct Ray {
    V o, d;
    float time;
};
RT_DEV V at(const Ray& r, float t) { return r.o + t * r.d; }  // ray.rs:28-30

// ---------------------------------------------------------------------------
// Philox4x32-10 per-(pixel, sample) stream (replaces rand::thread_rng)
// ---------------------------------------------------------------------------
// d counts the draws made; draw d is word d % 4 of Philox block d / 4, whose words not
// yet drawn wait in r0..r2 (the first is returned at once), so 6 registers stay live.
struct Rng {
    uint32_t sample, pixel, d;
    uint32_t r0, r1, r2;
};
RT_DEV void philox(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one v_mad_u64_u32 per product instead of v_mul_lo_u32 + v_mul_hi_u32 (same bits; C5 +5%,
        // C2 +1.3%, C3/C4 +0.5%; profiles/r04/experiments/philox_mad64_ab_*.log)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32), lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}
struct Key {
    uint32_t k0, k1;
};

// Inlined in every product unit (round 4, with the SLP vectorizer off: C1 +3%, C4 +4.6% over the
// out-of-line call the main unit used to make; profiles/r04/experiments/philox_inline_ab_*.log).
// RT_PHILOX_CALL builds the out-of-line form (the EXEC-join fixture, below).
#ifdef RT_PHILOX_CALL
__device__ __noinline__
#else
__device__ __forceinline__
#endif
uint4 philox_block(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t k0, uint32_t k1) {
    uint32_t c3 = 0u;
    philox(c0, c1, c2, c3, k0, k1);
    return make_uint4(c0, c1, c2, c3);
}
// RT_RNG_UNIFORM (the default when philox_block is an out-of-line call, RT_PHILOX_CALL): the
// block is computed under a wave-uniform branch (any active lane needs one) and taken per
// lane by select, so no divergent join carries the buffer. With the per-lane branch around
// the call, ROCm 7.2's VGPR allocator split the buffer's live ranges at the top of the join,
// ahead of its EXEC restore, so the copies moved r0 / r2 for the calling lanes only and the
// others' next draw was wrong (the C1 / C4 builds that left the oracle's bits).
// librtamd_rngdiv.so is that build, kept as the regression fixture of tools/exec_join_check.py,
// which tests/test_exec_join.py runs on every product build. The product inlines Philox (no
// call at the join) and keeps the per-lane branch, which measured 1-2% faster than the uniform
// form in the inlined units (C3, C5; rng_uniform_fix_ab_*.log).
#ifndef RT_RNG_UNIFORM
#ifdef RT_PHILOX_CALL
#define RT_RNG_UNIFORM 1
#else
#define RT_RNG_UNIFORM 0
#endif
#endif
RT_DEV uint32_t next_u32(Rng& g, const Key& k) {
#if RT_RNG_UNIFORM
    const bool fresh = (g.d & 3u) == 0u;
    uint32_t r = g.r0, r0 = g.r1, r1 = g.r2, r2 = g.r2;
    if (__ballot(fresh) != 0ull) {
        const uint4 b = philox_block(g.d >> 2, g.sample, g.pixel, k.k0, k.k1);
        r = fresh ? b.x : r;
        r0 = fresh ? b.y : r0;
        r1 = fresh ? b.z : r1;
        r2 = fresh ? b.w : r2;
    }
    g.r0 = r0; g.r1 = r1; g.r2 = r2;
#else
    uint32_t r;
    if ((g.d & 3u) == 0u) {
        const uint4 b = philox_block(g.d >> 2, g.sample, g.pixel, k.k0, k.k1);
        r = b.x;
        g.r0 = b.y; g.r1 = b.z; g.r2 = b.w;
    } else {
        r = g.r0;
        g.r0 = g.r1; g.r1 = g.r2;
    }
#endif
    g.d += 1u;
    return r;
}
RT_DEV float std01(Rng& g, const Key& k) {  // rand 0.8.5 Standard f32
    return (1.0f / 16777216.0f) * (float)(next_u32(g, k) >> 8);
}
RT_DEV float from_1_2(uint32_t u) { return __uint_as_float((u >> 9) | 0x3f800000u); }
// UniformFloat::sample_single for gen_range(-1.0..1.0) (utils.rs's only ranges on the path):
// v01 * scale + low with scale = 2, low = -1. Its retry (res >= high) never fires for this
// range: from_1_2(u) - 1 lies in [0, 1 - 2^-23], times 2 is exact, minus 1 gives
// [-1, 1 - 2^-22] exactly, always < 1; so one word is one value.
[[maybe_unused]] RT_DEV float range_pm1(uint32_t u) { return (from_1_2(u) - 1.0f) * 2.0f + -1.0f; }
#ifdef RT_SEQ_DRAWS
// Sequential draws (the EXEC-join regression fixture, librtamd_rngdiv.so, is built this way: the
// form of round 3 and early round 4, one next_u32 per coordinate with rand's retry loop).
RT_DEV float range_f(Rng& g, const Key& k, float low, float high) {  // UniformFloat::sample_single
    float scale = high - low;
    for (;;) {
        float v01 = from_1_2(next_u32(g, k)) - 1.0f;
        float res = v01 * scale + low;
        if (res < high) return res;
        scale = __uint_as_float(__float_as_uint(scale) - 1u);
    }
}
RT_DEV V in_unit_sphere(Rng& g, const Key& k) {  // materials/utils.rs:6-19
    for (;;) {
        float x = range_f(g, k, -1.0f, 1.0f);
        float y = range_f(g, k, -1.0f, 1.0f);
        float z = range_f(g, k, -1.0f, 1.0f);
        V v = mk(x, y, z);
        if (dot(v, v) < 1.0f) return v;
    }
}
RT_DEV V in_unit_disk(Rng& g, const Key& k) {  // utils.rs:9-17
    for (;;) {
        float x = range_f(g, k, -1.0f, 1.0f);
        float y = range_f(g, k, -1.0f, 1.0f);
        V p = mk(x, y, 0.0f);
        if (dot(p, p) < 1.0f) return p;
    }
}
#else
// gen_range(-1.0..1.0) never retries (range_pm1), so every attempt of in_unit_sphere takes
// exactly the words d, d+1, d+2 of the stream, at most one Philox block beyond the buffer:
// j = d % 4 = 0 -> block d/4 words 0-2; 1 -> the buffered words 1-3; 2 -> buffered 2, 3 and word 0
// of block d/4 + 1; 3 -> buffered 3 and words 0, 1 of the next block. The attempt computes that
// block once, under a wave-uniform branch, where three sequential draws ran Philox whenever any
// lane crossed a block boundary, i.e. up to three times per attempt for a wave whose lanes are
// out of phase. The words and the buffer it leaves are those of the sequential draws.
RT_DEV V in_unit_sphere(Rng& g, const Key& k) {  // materials/utils.rs:6-19
    for (;;) {
        const uint32_t j = g.d & 3u;
        uint4 b = make_uint4(g.r0, g.r1, g.r2, g.r2);
        if (__ballot(j != 1u) != 0ull) b = philox_block((g.d + 2u) >> 2, g.sample, g.pixel, k.k0, k.k1);
        const bool j0 = j == 0u, j1 = j == 1u, j2 = j == 2u;
        const uint32_t u0 = j0 ? b.x : g.r0;
        const uint32_t u1 = j0 ? b.y : (j1 || j2 ? g.r1 : b.x);
        const uint32_t u2 = j0 ? b.z : (j1 ? g.r2 : (j2 ? b.x : b.y));
        const uint32_t n0 = j0 ? b.w : (j1 ? g.r2 : (j2 ? b.y : b.z));
        const uint32_t n1 = j0 ? b.w : (j1 ? g.r2 : (j2 ? b.z : b.w));
        const uint32_t n2 = j1 ? g.r2 : b.w;
        g.r0 = n0;
        g.r1 = n1;
        g.r2 = n2;
        g.d += 3u;
        V v = mk(range_pm1(u0), range_pm1(u1), range_pm1(u2));
        if (dot(v, v) < 1.0f) return v;
    }
}
// The same for the lens disk's two words per attempt: j = 0 -> block d/4 words 0, 1; 1, 2 ->
// the buffered words; 3 -> buffered word 3 and word 0 of the next block.
RT_DEV V in_unit_disk(Rng& g, const Key& k) {  // utils.rs:9-17
    for (;;) {
        const uint32_t j = g.d & 3u;
        uint4 b = make_uint4(g.r0, g.r1, g.r2, g.r2);
        if (__ballot(j == 0u || j == 3u) != 0ull) b = philox_block((g.d + 1u) >> 2, g.sample, g.pixel, k.k0, k.k1);
        const bool j0 = j == 0u, j3 = j == 3u;
        const uint32_t u0 = j0 ? b.x : g.r0;
        const uint32_t u1 = j0 ? b.y : (j3 ? b.x : g.r1);
        const uint32_t n0 = j0 ? b.z : (j3 ? b.y : g.r2);
        const uint32_t n1 = j0 ? b.w : (j3 ? b.z : g.r2);
        const uint32_t n2 = j0 || j3 ? b.w : g.r2;
        g.r0 = n0;
        g.r1 = n1;
        g.r2 = n2;
        g.d += 2u;
        V p = mk(range_pm1(u0), range_pm1(u1), 0.0f);
        if (dot(p, p) < 1.0f) return p;
    }
}
#endif

// ---------------------------------------------------------------------------
// primitive tests: return the parameter t of the first valid root only
// ---------------------------------------------------------------------------
struct RayD {  // the f64 copy of a ray for sphere.rs:57-78, |d|^2 hoisted
    double ox, oy, oz, dx, dy, dz, a;
};
RT_DEV RayD to_d(const Ray& r) {
    RayD q;
    q.ox = r.o.x; q.oy = r.o.y; q.oz = r.o.z;
    q.dx = r.d.x; q.dy = r.d.y; q.dz = r.d.z;
    q.a = (q.dx * q.dx + q.dy * q.dy) + q.dz * q.dz;
    return q;
}

// sphere.rs:57-82 — quadratic in f64; both candidate roots (the reference computes
// the far root only when the near one is rejected: same IEEE values either way).
struct Roots {
    double r1, r2;
    bool ok;
};
RT_DEV Roots sphere_roots(f4 s, const RayD& q) {
    double ocx = q.ox - (double)s.x, ocy = q.oy - (double)s.y, ocz = q.oz - (double)s.z;
    double rad = (double)s.w;
    double half_b = (ocx * q.dx + ocy * q.dy) + ocz * q.dz;
    double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - rad * rad;
    double disc = half_b * half_b - q.a * c;
    Roots R;
    R.ok = !sign_negative_d(disc);
    double sq = __builtin_sqrt(disc);
    R.r1 = (-half_b - sq) / q.a;
    R.r2 = (-half_b + sq) / q.a;
    return R;
}
// sphere.rs:83-89 — near root unless outside [t_min, t_max], then the far root.
RT_DEV bool sphere_select(const Roots& R, float tmin, float tmax, float& t) {
    if (!R.ok) return false;
    double root = R.r1;
    if (root < (double)tmin || (double)tmax < root) {
        root = R.r2;
        if (root < (double)tmin || (double)tmax < root) return false;
    }
    t = (float)root;
    return true;
}
// f32 pretest of sphere.rs:57-68's f64 discriminant, for long top-level sphere runs.
// Evaluated in f32 from the same f32 inputs, every rounding of half_b^2 - a * c
// stays within 24 * 2^-24 * M of the exact value, M = half_b^2 + a * (|oc|^2 + r^2)
// (Cauchy-Schwarz bounds each dot product by |oc| |d|), and the f64 evaluation
// within ~2^-48 M of it. A value below -2^-16 M (256x that margin; M >= 2^-100 so
// that underflow cannot matter) therefore proves the f64 discriminant negative:
// the reference rejects the sphere (disc.is_sign_negative()). inf / NaN never reject.
RT_DEV bool sphere_surely_missed(f4 s, const Ray& r) {
    const float ocx = r.o.x - s.x, ocy = r.o.y - s.y, ocz = r.o.z - s.z;
    const float a = (r.d.x * r.d.x + r.d.y * r.d.y) + r.d.z * r.d.z;
    const float hb = (ocx * r.d.x + ocy * r.d.y) + ocz * r.d.z;
    const float oc2 = (ocx * ocx + ocy * ocy) + ocz * ocz;
    const float r2 = s.w * s.w;
    const float hb2 = hb * hb;
    const float disc = hb2 - a * (oc2 - r2);
    const float m = hb2 + a * (oc2 + r2);
    return m > 0x1p-100f && disc < -0x1p-16f * m;
}
// sphere.rs:49-103. Before dividing, spheres whose near root is certainly beyond
// t_max, or whose far root is certainly before t_min, are rejected: with the
// 2^-40 margin the rounded quotient provably lies on the same side, so the
// reference would reject both roots too ("division-free rejects").
RT_DEV bool sphere_t(f4 s, const RayD& q, float tmin, float tmax, float& t) {
    double ocx = q.ox - (double)s.x, ocy = q.oy - (double)s.y, ocz = q.oz - (double)s.z;
    double rad = (double)s.w;
    double half_b = (ocx * q.dx + ocy * q.dy) + ocz * q.dz;
    double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - rad * rad;
    double disc = half_b * half_b - q.a * c;
    if (sign_negative_d(disc)) return false;
    double sq = __builtin_sqrt(disc);
    double n1 = -half_b - sq, n2 = -half_b + sq;
    if (q.a > 0.0 && q.a < 1.0e300) {
        const double up = 1.0 + 0x1p-40, down = 1.0 - 0x1p-40;
        if (tmax > 0.0f && tmax < kInf && n1 > ((double)tmax * q.a) * up) return false;
        if (tmin > 0.0f && n2 < ((double)tmin * q.a) * down) return false;
    }
    double root = n1 / q.a;
    if (root < (double)tmin || (double)tmax < root) {
        root = n2 / q.a;
        if (root < (double)tmin || (double)tmax < root) return false;
    }
    t = (float)root;
    return true;
}

// moving_sphere.rs:47-51
RT_DEV V msphere_center(f4 m0, f4 m1, f4 m2, float time) {
    float s = (time - m1.w) / m2.x;
    return xyz(m0) + s * xyz(m1);
}
// moving_sphere.rs:54-84 — f32
RT_DEV bool msphere_t(f4 m0, f4 m1, f4 m2, const Ray& r, float tmin, float tmax, float& t) {
    V oc = r.o - msphere_center(m0, m1, m2, r.time);
    float a = dot(r.d, r.d);
    float half_b = dot(oc, r.d);
    float c = dot(oc, oc) - m0.w * m0.w;
    float disc = half_b * half_b - a * c;
    if (sign_negative(disc)) return false;
    float sq = __builtin_sqrtf(disc);
    float root = (-half_b - sq) / a;
    if (root < tmin || tmax < root) {
        root = (-half_b + sq) / a;
        if (root < tmin || tmax < root) return false;
    }
    t = root;
    return true;
}

// Division from a correctly rounded reciprocal (Markstein): with inv = RN(1/d), q0 = RN(x * inv),
// r = fma(-d, q0, x) (exact) and q = RN(q0 + r * inv) equals RN(x / d) whenever no intermediate under-
// or overflows and r is representable. Checked exhaustively over all 2^46 pairs of f32 significands
// (tools/markstein_check.hip, profiles/r05/markstein_check.log: 0 mismatches); scaling x and d by
// powers of two scales every step exactly. A cube leaf inside a BVH traversal has the ray's
// reciprocals at hand (bvh_hit's inv): when the scene's rect coordinates k (S.rect_rcp_ok) and the
// ray's origin components are +-0 or of magnitude in [2^-20, 2^20] and its direction components are
// in that range (rcp_ray_ok), x = k - o is 0 (never -0: no coordinate is -0) or of magnitude in
// [2^-43, 2^21], q0 lies in [2^-63, 2^41] or is a zero of the right sign, and r = x - d q0 is a
// multiple of at least 2^-149, hence exact: every side quotient is the reference's division.
#ifndef RT_MARKSTEIN_CUBE
#define RT_MARKSTEIN_CUBE 1
#endif
RT_DEV bool rcp_range(float v) {  // |v| in [2^-20, 2^20]
    return (__float_as_uint(v) & 0x7fffffffu) - 0x35800000u <= 0x49800000u - 0x35800000u;
}
RT_DEV bool rcp_ray_ok(const Ray& r) {
    const auto zero = [](float v) { return (__float_as_uint(v) & 0x7fffffffu) == 0u; };
    return rcp_range(r.d.x) && rcp_range(r.d.y) && rcp_range(r.d.z) && (zero(r.o.x) || rcp_range(r.o.x)) &&
           (zero(r.o.y) || rcp_range(r.o.y)) && (zero(r.o.z) || rcp_range(r.o.z));
}
RT_DEV float rcp_quotient(float k, float ok, float dk, float dinv) {  // (k - ok) / dk under the gate above
    const float x = k - ok, q0 = x * dinv;
    return __builtin_fmaf(__builtin_fmaf(-dk, q0, x), dinv, q0);
}
RT_DEV bool side_t_rcp(float k, float ok, float dk, float dinv, float oa, float da, float ob, float db, float a0,
                       float a1, float b0, float b1, float tmin, float tmax, float& t) {
    const float tt = rcp_quotient(k, ok, dk, dinv);
    if (tt < tmin || tt > tmax) return false;
    const float xx = oa + tt * da;
    const float yy = ob + tt * db;
    if (xx < a0 || xx > a1 || yy < b0 || yy > b1) return false;
    t = tt;
    return true;
}

// rectangle.rs:36-65 / 98-127 / 160-189; axis 0 = XY (plane z), 1 = XZ (plane y), 2 = YZ (plane x)
// Selects between values, never between addresses (a select of struct-member
// addresses pins the struct in scratch memory).
RT_DEV float sel3(uint32_t axis, float v0, float v1, float v2) { return axis == 0u ? v0 : (axis == 1u ? v1 : v2); }
RT_DEV void rect_axes(uint32_t axis, const Ray& r, float& ok, float& dk, float& oa, float& da, float& ob,
                      float& db) {
    const float ox = r.o.x, oy = r.o.y, oz = r.o.z, dx = r.d.x, dy = r.d.y, dz = r.d.z;
    ok = sel3(axis, oz, oy, ox);
    dk = sel3(axis, dz, dy, dx);
    oa = sel3(axis, ox, ox, oy);
    da = sel3(axis, dx, dx, dy);
    ob = sel3(axis, oy, oz, oz);
    db = sel3(axis, dy, dz, dz);
}
// rectangle.rs:36-65 with the plane axis resolved: k along (ok, dk), bounds
// [a0, a1] x [b0, b1] along (oa, da) x (ob, db). Same IEEE operations as rect_t.
RT_DEV bool side_t(float k, float ok, float dk, float oa, float da, float ob, float db, float a0, float a1, float b0,
                   float b1, float tmin, float tmax, float& t) {
    const float tt = (k - ok) / dk;
    if (tt < tmin || tt > tmax) return false;
    const float x = oa + tt * da;
    const float y = ob + tt * db;
    if (x < a0 || x > a1 || y < b0 || y > b1) return false;
    t = tt;
    return true;
}
RT_DEV bool rect_t(f4 r0, f4 r1, const Ray& r, float tmin, float tmax, float& t) {
    float ok, dk, oa, da, ob, db;
    rect_axes(__float_as_uint(r1.y), r, ok, dk, oa, da, ob, db);
    float tt = (r0.x - ok) / dk;
    if (tt < tmin || tt > tmax) return false;
    float x = oa + tt * da;
    float y = ob + tt * db;
    if (x < r0.y || x > r0.z || y < r0.w || y > r1.x) return false;
    t = tt;
    return true;
}

// triangle.rs:32-92 (Moller-Trumbore, eps 1e-7)
RT_DEV bool tri_t(f4 t0, f4 t1, f4 t2, const Ray& r, float tmin, float tmax, float& t) {
    const float eps = 0.0000001f;
    V e1 = xyz(t1), e2 = xyz(t2);
    V h = cross(r.d, e2);
    float a = dot(e1, h);
    if (a > -eps && a < eps) return false;
    float f = 1.0f / a;
    V s = r.o - xyz(t0);
    float u = f * dot(s, h);
    if (u < 0.0f || u > 1.0f) return false;
    V q = cross(s, e1);
    float v = f * dot(r.d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    float tt = f * dot(e2, q);
    if (tt < tmin || tt > tmax) return false;
    if (!(tt > eps)) return false;
    t = tt;
    return true;
}

// Scene features a fast-kernel instance is compiled for (kF): code for features a
// scene lacks is left out of its instance, since unused code still costs the
// instance registers and speed (measured: a flat scene runs 13% faster without
// the BVH code, showcase 2.5% faster without the triangle code).
// kFDeep: a BVH stack deeper than kStackLdsMax entries; kFLeafRM: BVH leaves that are
// rects or moving spheres (BVH leaf tests otherwise handle spheres, cubes, triangles).
constexpr uint32_t kFBvh = 1u, kFTri = 2u, kFRuns = 4u, kFDeep = 8u, kFLeafRM = 16u, kFMarble = 32u, kFAll = 63u;
// kFMarble: Marble textures, whose Perlin turbulence the whole wave evaluates together (turbulence_wave).
// kFSusp (a strategy, not a scene feature): the suspending list walk (world_walk), for the
// triangle-BVH preset, whose deep unpruned traversals ran at ~2 active lanes in their tails.
// Measured on the same box (50-spp frames): C4 197 -> 128 ms; the flat / sphere-BVH presets
// are 5-8% slower with it (C3 124 -> 133 ms, C5 152 -> 160 ms), so only that preset uses it.
constexpr uint32_t kFSusp = 64u;

[[maybe_unused]] constexpr uint32_t kStackLdsMax = 19u;  // LDS stack entries per lane at most (9.5 KB per wave: 16 waves/CU)
// The fast-kernel preset of a scene's features (fast_instance below).
constexpr uint32_t preset_of(uint32_t features) {
    return features == 0u                                        ? 0u
           : (features & ~kFRuns) == 0u                          ? kFRuns
           : (features & ~kFBvh) == 0u                           ? kFBvh
           : (features & ~(kFBvh | kFMarble)) == 0u              ? (kFBvh | kFMarble)
           : (features & ~(kFBvh | kFTri | kFDeep)) == 0u        ? (kFBvh | kFTri | kFDeep | kFSusp)
                                                                 : kFAll;
}
// One leaf (primitive or cube). tmax = closest so far; a hit with t == closest is
// accepted, so later candidates win ties exactly like hittable.rs:110-116.
// kTop: a top-level entry's primitive, at a wave-uniform address (ld4c: scalar loads)
template <bool kC>
RT_DEV f4 ldt(const f4* p) {
    if constexpr (kC) return ld4c(p);
    return ld4(p);
}
// RT_LEAF_EMBED: the BVH leaf test reads a leaf node's spheres (cx, cy, cz, r; lower.cpp
// repeats them in the free slot lanes) and its cubes' bounds (a cube's leaf box is exactly its
// bounds) from the node's own rows, so it no longer waits on a second, dependent load from sph /
// rect, nor holds those scene pointers across the traversal loop. 0 builds the round-5 leaf
// reads (A/B).
// The sphere-BVH presets only: the triangle preset's instance spilled 10 more VGPRs for code its
// scenes do not run.
#ifndef RT_LEAF_EMBED
#define RT_LEAF_EMBED 1
#endif
template <uint32_t kF>
constexpr bool kLeafEmbed = RT_LEAF_EMBED && (kF & kFTri) == 0u;
// cube.rs:84-93: the six sides as a HittableList. The sides' axes are fixed (cube.rs:25-74:
// xy z0, xy z1, xz y0, xz y1, yz x0, yz x1) and their bounds are the box's six values.
template <bool kInv>
RT_DEV bool cube_hit(const DevScene& S, uint32_t idx, float x0, float y0, float z0, float x1, float y1, float z1,
                     const Ray& r, V inv, float tmin, float& closest, uint32_t& hit_code) {
    const float ox = r.o.x, oy = r.o.y, oz = r.o.z, dx = r.d.x, dy = r.d.y, dz = r.d.z;
    float t;
    bool any = false;
    uint32_t face = 0u;
    if (kInv && RT_MARKSTEIN_CUBE && S.rect_rcp_ok && rcp_ray_ok(r)) {  // the ray's reciprocals (side_t_rcp)
        if (side_t_rcp(z0, oz, dz, inv.z, ox, dx, oy, dy, x0, x1, y0, y1, tmin, closest, t)) { closest = t; face = 0u; any = true; }
        if (side_t_rcp(z1, oz, dz, inv.z, ox, dx, oy, dy, x0, x1, y0, y1, tmin, closest, t)) { closest = t; face = 1u; any = true; }
        if (side_t_rcp(y0, oy, dy, inv.y, ox, dx, oz, dz, x0, x1, z0, z1, tmin, closest, t)) { closest = t; face = 2u; any = true; }
        if (side_t_rcp(y1, oy, dy, inv.y, ox, dx, oz, dz, x0, x1, z0, z1, tmin, closest, t)) { closest = t; face = 3u; any = true; }
        if (side_t_rcp(x0, ox, dx, inv.x, oy, dy, oz, dz, y0, y1, z0, z1, tmin, closest, t)) { closest = t; face = 4u; any = true; }
        if (side_t_rcp(x1, ox, dx, inv.x, oy, dy, oz, dz, y0, y1, z0, z1, tmin, closest, t)) { closest = t; face = 5u; any = true; }
    } else {
        if (side_t(z0, oz, dz, ox, dx, oy, dy, x0, x1, y0, y1, tmin, closest, t)) { closest = t; face = 0u; any = true; }
        if (side_t(z1, oz, dz, ox, dx, oy, dy, x0, x1, y0, y1, tmin, closest, t)) { closest = t; face = 1u; any = true; }
        if (side_t(y0, oy, dy, ox, dx, oz, dz, x0, x1, z0, z1, tmin, closest, t)) { closest = t; face = 2u; any = true; }
        if (side_t(y1, oy, dy, ox, dx, oz, dz, x0, x1, z0, z1, tmin, closest, t)) { closest = t; face = 3u; any = true; }
        if (side_t(x0, ox, dx, oy, dy, oz, dz, y0, y1, z0, z1, tmin, closest, t)) { closest = t; face = 4u; any = true; }
        if (side_t(x1, ox, dx, oy, dy, oz, dz, y0, y1, z0, z1, tmin, closest, t)) { closest = t; face = 5u; any = true; }
    }
    if (any) hit_code = rtdev::leaf_code(rtdev::kLeafRect, idx + face);
    return any;
}
// kNoSphCube: the caller has tested sphere and cube leaves itself (bvh_run, RT_LEAF_EMBED).
template <uint32_t kF = kFAll, bool kInv = false, bool kTop = false, bool kNoSphCube = false>
RT_DEV bool leaf_hit(const DevScene& S, uint32_t code, const Ray& r, const RayD& q, float tmin, float& closest,
                     uint32_t& hit_code, V inv = V{0.0f, 0.0f, 0.0f}) {
    uint32_t type = rtdev::leaf_type(code), idx = rtdev::leaf_index(code);
    float t;
    if (!kNoSphCube && type == rtdev::kLeafSphere) {
        if (sphere_t(ldt<kTop>(S.sph + idx), q, tmin, closest, t)) {
            closest = t;
            hit_code = code;
            return true;
        }
        return false;
    }
    if ((kF & kFLeafRM) && type == rtdev::kLeafRect) {
        if (rect_t(ldt<kTop>(S.rect + 2 * idx), ldt<kTop>(S.rect + 2 * idx + 1), r, tmin, closest, t)) {
            closest = t;
            hit_code = code;
            return true;
        }
        return false;
    }
    if (!kNoSphCube && type == rtdev::kLeafCube) {
        // the bounds from the records of sides 0 and 2: (z0, x0, x1, y0), y1 and (y0, x0, x1, z0), z1
        const f4 s0 = ldt<kTop>(S.rect + 2 * idx);
        const float y1 = ldt<kTop>(S.rect + 2 * idx + 1).x, z1 = ldt<kTop>(S.rect + 2 * idx + 5).x;
        return cube_hit<kInv>(S, idx, s0.y, s0.w, s0.x, s0.z, y1, z1, r, inv, tmin, closest, hit_code);
    }
    if ((kF & kFTri) && type == rtdev::kLeafTri) {
        if (tri_t(ldt<kTop>(S.tri + 3 * idx), ldt<kTop>(S.tri + 3 * idx + 1), ldt<kTop>(S.tri + 3 * idx + 2), r, tmin, closest, t)) {
            closest = t;
            hit_code = code;
            return true;
        }
        return false;
    }
    if ((kF & kFLeafRM) && type == rtdev::kLeafMSphere) {
        if (msphere_t(ldt<kTop>(S.msph + 3 * idx), ldt<kTop>(S.msph + 3 * idx + 1), ldt<kTop>(S.msph + 3 * idx + 2), r, tmin, closest,
                      t)) {
            closest = t;
            hit_code = code;
            return true;
        }
    }
    return false;
}

// aabb.rs:28-41 (Kensler). 1/d is hoisted per ray: the same IEEE quotient the
// reference recomputes per node. All three slabs are evaluated branch-free; the
// interval only shrinks, so this equals the reference's early-exit result.
// t_enter receives the final t_min (the ray's entry parameter into the box).
RT_DEV bool slab(float x0, float y0, float z0, float x1, float y1, float z1, const Ray& r, V inv, float t_min,
                 float t_max, float& t_enter) {
    {
        float t0 = (x0 - r.o.x) * inv.x, t1 = (x1 - r.o.x) * inv.x;
        bool sw = inv.x < 0.0f;
        float a = sw ? t1 : t0, b = sw ? t0 : t1;
        t_min = a > t_min ? a : t_min;
        t_max = b < t_max ? b : t_max;
    }
    {
        float t0 = (y0 - r.o.y) * inv.y, t1 = (y1 - r.o.y) * inv.y;
        bool sw = inv.y < 0.0f;
        float a = sw ? t1 : t0, b = sw ? t0 : t1;
        t_min = a > t_min ? a : t_min;
        t_max = b < t_max ? b : t_max;
    }
    {
        float t0 = (z0 - r.o.z) * inv.z, t1 = (z1 - r.o.z) * inv.z;
        bool sw = inv.z < 0.0f;
        float a = sw ? t1 : t0, b = sw ? t0 : t1;
        t_min = a > t_min ? a : t_min;
        t_max = b < t_max ? b : t_max;
    }
    t_enter = t_min;
    return !(t_max < t_min);
}

// A subtree may be skipped once its inflated entry exceeds this bound: every
// candidate inside it would then compute t > closest (exact pruning).
RT_DEV float prune_bound(float closest) { return closest + __builtin_fabsf(closest) * 0x1p-19f; }

// Conservative leaf test (prunable BVHs only, leaf_intervals2_nf +
// leaf_interval_may_hit): false only when the leaf's primitive provably has no hit
// in [tmin, closest]. The box is the primitive's own bounding box inflated by
// delta; any computed hit t lies on the ray within rounding distance (<< delta) of
// that box, and the slab values carry <= 3 relative roundings, so the 2^-19
// slacks cover them ("exact pruning").

// Bvh::hit / BvhNode::hit (bvh.rs:212-217, 363-417) as an iterative traversal of
// BVH2 nodes. Every child box gets the reference's own test (stored box, the
// t_max the BVH was entered with), so no node outside the reference's visit set
// is ever entered. For BVHs flagged kBvhPrunable (f64 spheres / rects / cubes)
// a visited subtree is additionally skipped when its entry into the box
// inflated by P.prune_delta lies beyond prune_bound(closest), and a leaf is
// skipped when its own inflated box rules out a hit in [tmin, closest]: such
// candidates provably cannot beat (closest, rank). Children are visited
// nearest-first; ties resolve by DFS rank exactly like the recursion.
// The stack lives in LDS, lane-strided: stack[level * 128 + {0, 64} + lane].
#ifdef RT_LEAF_AUDIT
// Leaf-box audit (audit build): a leaf rejected by the conservative test is tested
// anyway, and recorded if it would have produced a candidate.
#define LEAF_AUDIT(CODE_, RANK_, X0_, Y0_, Z0_, X1_, Y1_, Z1_)                                          \
    do {                                                                                               \
        float c_ = tmax_entry;                                                                         \
        uint32_t hc_ = 0u;                                                                             \
        if (leaf_hit(S, (CODE_), r, to_d(r), tmin, c_, hc_) && !(c_ > bound)) {                              \
            unsigned i_ = atomicAdd(&g_audit_count, 1u);                                               \
            if (i_ < kAuditMax) {                                                                      \
                LeafAudit& A = g_audit[i_];                                                            \
                A.o[0] = r.o.x; A.o[1] = r.o.y; A.o[2] = r.o.z;                                        \
                A.d[0] = r.d.x; A.d[1] = r.d.y; A.d[2] = r.d.z;                                        \
                A.tmin = tmin; A.closest = closest; A.t = c_; A.delta = delta;                         \
                A.box[0] = (X0_); A.box[1] = (Y0_); A.box[2] = (Z0_);                                  \
                A.box[3] = (X1_); A.box[4] = (Y1_); A.box[5] = (Z1_);                                  \
                A.code = (CODE_); A.rank = (RANK_); A.best_rank = hc_;                                 \
            }                                                                                          \
        }                                                                                              \
    } while (0)
#else
#define LEAF_AUDIT(CODE_, RANK_, X0_, Y0_, Z0_, X1_, Y1_, Z1_) do { } while (0)
#endif
// BvhNode::hit (bvh.rs:363-417) replayed literally on the reference BVH2: the
// node's box with the BVH's entry t_max, the left child (an Index child with
// t_max, a Hittable with t_max), then the right child (an Index child with
// t_max, a Hittable with the left hit's t), and `if left.t < right.t {left}
// else {right}`. The reference kernel (trace_samples<1>) traverses every BVH
// this way: RT_FLAG_EXACT_BVH renders, and the samples the fast kernel hands
// over because one of their rays could take a NaN hit (with a NaN t in play the
// tree-min is neither associative nor order-independent, so only the
// reference's own recursion order is exact).
// One frame per level: stk[level * 256 + {0, 64, 128, 192} + lane] = node,
// phase | left-hit << 2, left t, left code. Phases: 0 start, 1 waiting for the
// left subtree, 2 left known, 3 waiting for the right subtree.
RT_DEV bool bvh_hit_reference(const DevScene& S, uint32_t wrapper2, const Ray& r, const RayD& q, V inv, float tmin,
                              float& closest, uint32_t& hit_code, uint32_t* stk) {
    const float tmax = closest;
    const f4* w = S.nodes2 + 4 * (size_t)wrapper2;
    const f4 w3 = ld4(w + 3);
    if ((__float_as_uint(w3.w) & rtdev::kBvh2TriOnly) &&
        (r.o.x != r.o.x || r.o.y != r.o.y || r.o.z != r.o.z || r.d.x != r.d.x || r.d.y != r.d.y || r.d.z != r.d.z))
        return false;  // no triangle takes a NaN ray (device_scene.hpp kBvh2TriOnly): the recursion's answer
    {
        f4 w0 = ld4(w), w1 = ld4(w + 1);
        float te;
        if (!slab(w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, r, inv, tmin, tmax, te)) return false;  // bvh.rs:370
    }
    uint32_t sp = 1u;
    stk[0] = __float_as_uint(w3.x);
    stk[64] = 0u;
    bool rh = false, returning = false;
    float rt = 0.0f;
    uint32_t rcode = 0u;
    for (;;) {
        uint32_t* F = stk + (sp - 1u) * 256u;
        uint32_t st = F[64];
        if (returning) {  // deliver the finished child's result to its parent frame
            if ((st & 3u) == 1u) {
                F[64] = 2u | (rh ? 4u : 0u);
                F[128] = __float_as_uint(rt);
                F[192] = rcode;
                returning = false;
                continue;
            }
            // phase 3: right subtree done -> combine with the stored left result
            if ((st & 4u) && !(rh && !(__uint_as_float(F[128]) < rt))) {
                rt = __uint_as_float(F[128]);
                rcode = F[192];
                rh = true;
            }
            sp -= 1u;
            if (sp == 0u) break;
            continue;
        }
#ifdef RT_LEAF_AUDIT
        if (F[0] >= S.num_nodes2 || 2u * sp > S.stack_depth) {  // a frame is two 128-word stack entries
            atomicAdd(&g_bounds_audit_count, 1u);
            break;
        }
#endif
        const f4* nd = S.nodes2 + 4 * (size_t)F[0];
        f4 n0 = ld4(nd), n1 = ld4(nd + 1), n2 = ld4(nd + 2), n3 = ld4(nd + 3);
        const uint32_t lc = __float_as_uint(n3.x), rc = __float_as_uint(n3.y);
        if ((st & 3u) == 0u) {  // left child
            if (lc & rtdev::kLeafBit) {
                float c = tmax;
                uint32_t code = 0u;
                bool h = leaf_hit(S, lc, r, q, tmin, c, code);
                F[64] = 2u | (h ? 4u : 0u);
                F[128] = __float_as_uint(c);
                F[192] = code;
            } else {
                float te;
                if (slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, r, inv, tmin, tmax, te)) {
                    F[64] = 1u;
                    stk[sp * 256u] = lc;
                    stk[sp * 256u + 64u] = 0u;
                    sp += 1u;
                } else {
                    F[64] = 2u;
                }
            }
            continue;
        }
        // phase 2: right child (a 1-object node repeats its left object: same result)
        const bool hl = (st & 4u) != 0u;
        const float tl = __uint_as_float(F[128]);
        if (rc == rtdev::kChildEmpty || (rc & rtdev::kLeafBit)) {
            float c = hl ? tl : tmax;  // t_max_for_right
            uint32_t code = 0u;
            bool hr = rc != rtdev::kChildEmpty && leaf_hit(S, rc, r, q, tmin, c, code);
            if (hr && !(hl && tl < c)) {
                rh = true;
                rt = c;
                rcode = code;
            } else {
                rh = hl;
                rt = tl;
                rcode = F[192];
            }
            sp -= 1u;
            if (sp == 0u) break;
            returning = true;
            continue;
        }
        float te;
        if (slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, r, inv, tmin, tmax, te)) {
            F[64] = 3u | (st & 4u);
            stk[sp * 256u] = rc;
            stk[sp * 256u + 64u] = 0u;
            sp += 1u;
        } else {  // no right hit: the left result stands
            rh = hl;
            rt = tl;
            rcode = F[192];
            sp -= 1u;
            if (sp == 0u) break;
            returning = true;
        }
    }
    if (rh) {
        closest = rt;
        hit_code = rcode;
    }
    return rh;
}

// ---------------------------------------------------------------------------
// HRPP experiment (RT_FLAG_HRPP): hash-based ray path prediction, src/hrpp.rs +
// src/bvh.rs:114-211. Approximate by design; never on the parity path.
// ---------------------------------------------------------------------------
// hrpp.rs:136-170, BitPrecision::Six: sign | top 6 exponent bits | top 6 mantissa bits.
RT_DEV uint32_t hrpp_map_float(float v) {
    const uint32_t b = __float_as_uint(v);
    return ((b >> 31) << 15) | (((b >> 25) & 0x3fu) << 7) | ((b >> 17) & 0x3fu);
}
// hrpp.rs:172-193: the ray passed to Bvh::hit (its frame, unnormalised direction).
RT_DEV unsigned long long hrpp_hash(const Ray& r) {
    const unsigned long long h0 = hrpp_map_float(r.o.x) ^ hrpp_map_float(r.d.z);
    const unsigned long long h1 = hrpp_map_float(r.o.y) ^ hrpp_map_float(r.d.y);
    const unsigned long long h2 = hrpp_map_float(r.o.z) ^ hrpp_map_float(r.d.x);
    return h0 | (h1 << 16) | (h2 << 32);
}
// Open addressing, linear probing (32 probes); the slot's key is claimed by CAS.
RT_DEV rtdev::HrppSlot* hrpp_find(rtdev::HrppSlot* tab, uint32_t bits, unsigned long long key, bool insert) {
    const uint32_t mask = (1u << bits) - 1u;
    unsigned long long m = key * 0x9E3779B97F4A7C15ull;
    const uint32_t h = (uint32_t)(m >> 32) ^ (uint32_t)m;
    for (uint32_t i = 0; i < 32u; ++i) {
        rtdev::HrppSlot* sl = tab + ((h + i) & mask);
        unsigned long long k = __hip_atomic_load(&sl->key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return sl;
        if (k == ~0ull) {
            if (!insert) return nullptr;
            k = atomicCAS(&sl->key, ~0ull, key);
            if (k == ~0ull || k == key) return sl;
        }
    }
    return nullptr;
}
RT_DEV uint32_t hrpp_leaf_node(const DevScene& S, unsigned long long k) {  // sorted-map lookup
    uint32_t lo = 0, hi = S.hrpp_nkeys;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (S.hrpp_keys[m] < k) lo = m + 1;
        else hi = m;
    }
    return lo < S.hrpp_nkeys && S.hrpp_keys[lo] == k ? S.hrpp_vals[lo] : 0xffffffffu;
}
// Bvh::hit with a predictor (bvh.rs:120-211, GO_UP_LEVEL = 0). Counters per wave
// in LDS: true positive, false positive, no prediction, dropped insertions.
RT_DEV bool bvh_hit_hrpp(const DevScene& S, uint32_t wrapper2, uint32_t pid, const Ray& r,
                                          const RayD& q, V inv, float tmin, float& closest, uint32_t& hit_code,
                                          uint32_t* stk) {
    rtdev::HrppSlot* tab = S.hrpp_tab + ((size_t)(pid - 1u) << S.hrpp_bits);
    uint32_t* cnt = S.hrpp_cnt + 4u * (pid - 1u);
    const unsigned long long key = hrpp_hash(r);
    const rtdev::HrppSlot* sl = S.hrpp_bits ? hrpp_find(tab, S.hrpp_bits, key, false) : nullptr;
    bool predicted = false;
    if (sl) {  // bvh.rs:141-173: the closest hit among the predicted nodes
        float c = closest;
        uint32_t code = 0u;
        bool any = false;
        for (uint32_t j = 0; j < rtdev::kHrppIds; ++j) {
            const uint32_t w = __hip_atomic_load(&sl->ids[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (w == 0xffffffffu) break;
            predicted = true;
            if (bvh_hit_reference(S, w, r, q, inv, tmin, c, code, stk)) any = true;
        }
        if (any) {  // true positive: traversal skipped (possibly not the closest hit)
            atomicAdd(&cnt[0], 1u);
            closest = c;
            hit_code = code;
            return true;
        }
    }
    atomicAdd(&cnt[predicted ? 1u : 2u], 1u);  // false positive / no prediction: full traversal
    const bool h = bvh_hit_reference(S, wrapper2, r, q, inv, tmin, closest, hit_code, stk);
    if (h && S.hrpp_bits) {  // predictor.insert(ray, leaf node), bvh.rs:188-205
        const uint32_t leaf = hrpp_leaf_node(S, (unsigned long long)wrapper2 << 32 | hit_code);
        rtdev::HrppSlot* ins = leaf != 0xffffffffu ? hrpp_find(tab, S.hrpp_bits, key, true) : nullptr;
        bool ok = false;
        if (ins)
            for (uint32_t j = 0; j < rtdev::kHrppIds && !ok; ++j) {
                const uint32_t old = atomicCAS(&ins->ids[j], 0xffffffffu, leaf);
                ok = old == 0xffffffffu || old == leaf;
            }
        if (!ok) atomicAdd(&cnt[3], 1u);
    }
    return h;
}

// One interior child of a BVH4 node: the reference's box test (stored box, the
// t_max the BVH was entered with) and, when pruning, the inflated-entry bound.
// Returns the sort key: the entry distance, +inf when the child is not visited.
// The inflated entry is bounded from the reference test's own entry: along axis
// a the delta shell is delta * |inv_a| thick in t, so entry(box + delta) >=
// entry(box) - delta * max_a |inv_a| (= te - dmi). The gap to any candidate in
// the box stays >= delta / |d|, which dominates the slab roundings exactly as in
// the direct computation (exact pruning); a large dmi only weakens
// the bound (no pruning), never strengthens it.
// The returned key is what the stack keeps for the pop-time prune, so for a
// prunable BVH it is always the conservative (inflated) entry, also while
// closest is still infinite.
[[maybe_unused]] RT_DEV float child_key(float x0, float y0, float z0, float x1, float y1, float z1, const Ray& r, V inv, float tmin,
                       float tmax_entry, float closest, bool prune, float dmi) {
    float te;
    bool go = slab(x0, y0, z0, x1, y1, z1, r, inv, tmin, tmax_entry, te);
    if (prune) te = te - dmi;
    if (go && prune) go = !(te > prune_bound(closest));
    return go ? (te < 3.4028235e38f ? te : 3.4028235e38f) : kInf;  // visited children sort first
}
// child_key for all four slots of a node at once, on two children per packed
// f32 instruction (v_pk_add_f32 / v_pk_mul_f32: the same correctly rounded IEEE
// operations per element). The rows come ordered by the ray's direction signs (bvh_run
// loads them so): n* hold each axis's near plane (the max plane when 1/d < 0, aabb.rs:33-35's
// swap), f* the far one, so each slab value is the reference's (plane - o) * inv and no
// per-child select is left. Valid only without NaN slab values: the fast kernel
// replays every ray with a zero or non-finite 1/d component, so (plane - o) * inv
// is finite or +-inf, never 0 * inf, and the reference's sequential
// `if a > t_min {a} else {t_min}` clamps (aabb.rs:28-41) equal max/min. Empty
// slots hold an inverted infinite box (lower.cpp) and never pass. dmi = 0 and
// pb = +inf when the BVH is not prunable.
typedef float pk2 __attribute__((ext_vector_type(2)));
RT_DEV pk2 pk(float a, float b) { return pk2{a, b}; }
RT_DEV void child_keys4_nf(f4 nx, f4 ny, f4 nz, f4 fx, f4 fy, f4 fz, const Ray& r, V inv, float tmin,
                           float tmax_entry, float pb, float dmi, float key[4]) {
    const pk2 ox = pk(r.o.x, r.o.x), oy = pk(r.o.y, r.o.y), oz = pk(r.o.z, r.o.z);
    const pk2 ix = pk(inv.x, inv.x), iy = pk(inv.y, inv.y), iz = pk(inv.z, inv.z);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const pk2 tnx = ((h ? pk(nx.z, nx.w) : pk(nx.x, nx.y)) - ox) * ix, tfx = ((h ? pk(fx.z, fx.w) : pk(fx.x, fx.y)) - ox) * ix;
        const pk2 tny = ((h ? pk(ny.z, ny.w) : pk(ny.x, ny.y)) - oy) * iy, tfy = ((h ? pk(fy.z, fy.w) : pk(fy.x, fy.y)) - oy) * iy;
        const pk2 tnz = ((h ? pk(nz.z, nz.w) : pk(nz.x, nz.y)) - oz) * iz, tfz = ((h ? pk(fz.z, fz.w) : pk(fz.x, fz.y)) - oz) * iz;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float lo = __builtin_fmaxf(__builtin_fmaxf(tnx[e], tny[e]), __builtin_fmaxf(tnz[e], tmin));
            const float hi = __builtin_fminf(__builtin_fminf(tfx[e], tfy[e]), __builtin_fminf(tfz[e], tmax_entry));
            const float te = lo - dmi;
            const bool go = lo <= hi && te <= pb;  // = !(hi < lo) && !(te > pb) without NaN
            key[2 * h + e] = go ? __builtin_fminf(te, 3.4028235e38f) : kInf;
        }
    }
}
// The two leaf slots of a leaf node: the slab interval of each leaf's box inflated by
// delta, both leaves per packed instruction, on sign-ordered rows like child_keys4_nf. The
// inflation is folded into shifted origins: x0 - (o + delta) for a min plane, x1 - (o - delta)
// for a max one, with the error structure of (x0 - delta) - o (one rounding of a
// coordinate-sized value, <= 2^-24 R << delta, then relative roundings). NaN-free under the
// same 1/d condition as child_keys4_nf; an empty second slot (inverted infinite box) gives
// lo = +inf.
RT_DEV void leaf_intervals2_nf(float2 nx, float2 ny, float2 nz, float2 fx, float2 fy, float2 fz, const Ray& r,
                               V inv, float delta, float lo[2], float hi[2]) {
    const bool sx = inv.x < 0.0f, sy = inv.y < 0.0f, sz = inv.z < 0.0f;
    const float pxs = r.o.x + delta, pys = r.o.y + delta, pzs = r.o.z + delta;
    const float mxs = r.o.x - delta, mys = r.o.y - delta, mzs = r.o.z - delta;
    const float anx = sx ? mxs : pxs, afx = sx ? pxs : mxs, sny = sy ? mys : pys, afy = sy ? pys : mys;
    const float anz = sz ? mzs : pzs, afz = sz ? pzs : mzs;
    const pk2 ix = pk(inv.x, inv.x), iy = pk(inv.y, inv.y), iz = pk(inv.z, inv.z);
    const pk2 tnx = (pk(nx.x, nx.y) - pk(anx, anx)) * ix, tfx = (pk(fx.x, fx.y) - pk(afx, afx)) * ix;
    const pk2 tny = (pk(ny.x, ny.y) - pk(sny, sny)) * iy, tfy = (pk(fy.x, fy.y) - pk(afy, afy)) * iy;
    const pk2 tnz = (pk(nz.x, nz.y) - pk(anz, anz)) * iz, tfz = (pk(fz.x, fz.y) - pk(afz, afz)) * iz;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        lo[e] = __builtin_fmaxf(__builtin_fmaxf(tnx[e], tny[e]), tnz[e]);
        hi[e] = __builtin_fminf(__builtin_fminf(tfx[e], tfy[e]), tfz[e]);
    }
}
// The conservative leaf test's decision on a precomputed inflated interval.
RT_DEV bool leaf_interval_may_hit(float lo, float hi, float tmin, float closest) {
    if (lo > prune_bound(closest)) return false;
    if (tmin > 0.0f && hi < tmin * (1.0f - 0x1p-19f)) return false;
    return !(lo - hi > (__builtin_fabsf(lo) + __builtin_fabsf(hi)) * 0x1p-19f);
}
RT_DEV void sort2(float& ta, uint32_t& ca, float& tb, uint32_t& cb) {  // branch-free compare-exchange
    const bool sw = tb < ta;
    const float a = ta, b = tb;
    const uint32_t x = ca, y = cb;
    ta = sw ? b : a;
    tb = sw ? a : b;
    ca = sw ? y : x;
    cb = sw ? x : y;
}
// kKind 0: the fast BVH4 kernel; 1: the reference kernel replays bvh.rs literally;
// 2: the reference kernel with HRPP predictors (RT_FLAG_HRPP experiment); 3: the replay
// pass, fast traversal for every ray the fast kernel can take and the literal replay for
// the others, so a handed-over sample's other bounces run at fast speed. The fast kernel
// returns with `replay` set for a ray that could take a NaN hit: a ray parallel
// to an axis plane (a zero direction component) gets t = (k - o) / d = 0 / 0 from
// a rect whose plane holds its origin, and every comparison against NaN passes
// (rectangle.rs:36-65); its sample is re-traced by the reference kernel.
// A BVH traversal's state between visits (bvh_run).
struct Trav {
    uint32_t cur, sp, best_rank;
    float tmax_entry;
    bool any;
    uint32_t pend;  // a leaf node reached and not yet tested (kNoNode: none; bvh_run)
};
constexpr uint32_t kNoNode = 0xffffffffu;
// Audit build: every completed fast traversal is replayed with the reference recursion
// (bvh_hit_reference, on the lane's now free LDS stack); disagreements are recorded.
RT_DEV void trav_audit(const DevScene& S, const f4* wrapper, uint32_t root, const Ray& r, V inv, float tmin,
                       const Trav& tv, float closest, uint32_t hit_code, uint32_t* stk) {
#ifdef RT_LEAF_AUDIT
    const bool any = tv.any;
    float c2 = tv.tmax_entry;
    uint32_t h2 = 0u;
    bool a2 = bvh_hit_reference(S, __float_as_uint(ld4c(wrapper + 7).z), r, to_d(r), inv, tmin, c2, h2, stk);
    bool same = a2 == any && (!any || (__float_as_uint(c2) == __float_as_uint(closest) && h2 == hit_code));
    if (!same) {
        unsigned i_ = atomicAdd(&g_trav_audit_count, 1u);
        if (i_ < kAuditMax) {
            TravAudit& A = g_trav_audit[i_];
            A.o[0] = r.o.x; A.o[1] = r.o.y; A.o[2] = r.o.z;
            A.d[0] = r.d.x; A.d[1] = r.d.y; A.d[2] = r.d.z;
            A.tmin = tmin; A.tmax = tv.tmax_entry;
            A.fast_t = any ? closest : kInf; A.ref_t = a2 ? c2 : kInf;
            A.fast_code = any ? hit_code : 0xffffffffu; A.ref_code = a2 ? h2 : 0xffffffffu;
            A.root = root;
        }
    }
#endif
}
// The suspending walk lets a traversal stop only after this many visits in one call.
#ifndef RT_SUSP_MIN_TRIPS
#define RT_SUSP_MIN_TRIPS 2
#endif
constexpr uint32_t kSuspMinTrips = RT_SUSP_MIN_TRIPS;
#ifndef RT_LEAF_Q
#define RT_LEAF_Q 8
#endif

template <int kKind, uint32_t kF, bool kSusp>
RT_DEV bool bvh_run(const DevScene& S, float delta, const f4* wrapper, const Ray& r, V inv, float tmin, float& closest,
                    uint32_t& hit_code, uint32_t* stk, uint32_t mode, Trav& tv, uint32_t susp);
// Which traversal a ray takes into a BVH (bvh_hit, world_walk, the replay pass).
// kRayFast: the fast BVH4 traversal is exact for it. Its packed slab test (child_keys4_nf)
// forms each child's interval with max / min, and those equal aabb.rs:28-41's sequential
// `if t0 > t_min {t0} else {t_min}` clamps as long as the only NaN slab values are the ones the
// reference's comparisons ignore too: maxnum / minnum return the other operand of a quiet NaN,
// and the reference keeps t_min / t_max unchanged on a NaN t0 / t1; the empty slots' infinite
// planes must never give NaN, and the entry t_max must not be NaN (every reference box test
// passes with t_max = NaN, and HittableList::hit still takes the BVH's hit). So:
// * every BVH: a finite origin, 0 < |1/d| < inf on every axis (no NaN slab value at all, and
//   delta * max|1/d| stays finite for the exact-pruning margin), and a non-NaN entry t_max;
// * a triangle-only BVH (kBvhTriOnly: never prunable, no delta margin, and Tri::hit never
//   returns a NaN t): also a zero or denormal direction component. Then 1/d = +-inf and the only
//   NaN slab values are 0 * inf on a plane through the origin; the empty slots' planes give
//   (+-inf - o) * +-inf = +-inf. Round 5 handed these rays over (C4: ~15,500 samples a frame,
//   whose re-traced paths were the 23-50 ms replay tail).
// kRayNoHit: a triangle-only BVH and a NaN in the ray: Moller-Trumbore (triangle.rs:32-92) takes
// no such ray (a NaN reaches t and !(t > EPSILON) rejects it), so the BVH returns no hit whatever
// its boxes do (bvh_hit_reference's kBvh2TriOnly answer, without the walk).
// kRayHandOver: everything else goes to the literal recursion (a zero direction component in a
// BVH with rects, whose 0/0 = NaN hits make the tree-min order-dependent; a non-finite origin or
// direction; a NaN closest_so_far, e.g. from a 0/0 rect hit earlier in the list whose plane axis
// the BVH's own frame rotated away).
constexpr uint32_t kRayFast = 0u, kRayHandOver = 1u, kRayNoHit = 2u;
// Where: the relaxed rule for triangle-only BVHs is compiled into the replay pass (kKind 3), which
// re-traces handed-over samples from their camera ray, and (RT_TRI_ZERO_DIR_FAST 1, the default)
// into the fast kernel. In the fast kernel's 4-wave triangle instance the code cost 10% (C4 50 spp
// 62.0 vs 68.8 ms, profiles/r06/experiments/ray_route_zero_direction_ab.log); in the spill-free
// 3-wave instance the product runs since, it costs 0.7% of the fast kernel and removes C4's
// handed-over samples, whose re-traced paths ended 0-25 ms after the fast kernel (full C4 frame
// 1113 ms every run against 1111-1137 ms, profiles/r06/experiments/zero_direction_fast_kernel_ab.log).
// 0 builds the replay-pass-only rule (A/B).
#ifndef RT_TRI_ZERO_DIR_FAST
#define RT_TRI_ZERO_DIR_FAST 1
#endif
template <int kKind, uint32_t kF>
RT_DEV uint32_t ray_route(const Ray& r, V inv, float tmax_entry, const f4* wrapper, uint32_t mode) {
    const float ax = __builtin_fabsf(inv.x), ay = __builtin_fabsf(inv.y), az = __builtin_fabsf(inv.z);
    const bool ofin = __builtin_fabsf(r.o.x) < kInf && __builtin_fabsf(r.o.y) < kInf && __builtin_fabsf(r.o.z) < kInf;
    const bool tnum = tmax_entry == tmax_entry;
    if (ax > 0.0f && ax < kInf && ay > 0.0f && ay < kInf && az > 0.0f && az < kInf && ofin && tnum) return kRayFast;
    if constexpr ((kF & kFTri) != 0u && (kKind == 3 || (kKind == 0 && RT_TRI_ZERO_DIR_FAST))) {
        if ((__float_as_uint(ld4c(wrapper + 7).w) & rtdev::kBvhTriOnly) != 0u &&
            !(kPruneAllExpBuild && (mode & kModePruneAllExp))) {
            if (r.o.x != r.o.x || r.o.y != r.o.y || r.o.z != r.o.z || r.d.x != r.d.x || r.d.y != r.d.y ||
                r.d.z != r.d.z)
                return kRayNoHit;
            const bool dfin =
                __builtin_fabsf(r.d.x) < kInf && __builtin_fabsf(r.d.y) < kInf && __builtin_fabsf(r.d.z) < kInf;
            if (dfin && ofin && tnum) return kRayFast;
        }
    }
    return kRayHandOver;
}

// A triangle-only BVH entered with a NaN closest_so_far, in the replay pass (bvh_hit, kKind 3), for a
// ray with a finite origin and direction. With t_max = NaN every reference box test passes
// (aabb.rs:28-41: `t1 < t_max` and `t_max <= t_min` are false), and BvhNode::hit (bvh.rs:363-417)
// passes its own t_max to both Index children (only a leaf's right object gets the left object's t),
// so the t_max stays NaN on every level: every leaf node is visited and the tree keeps, by
// `if l.t < r.t {l} else {r}`, the least t with ties going to the later object in DFS order. A leaf
// node's left object is tested against NaN (Moller-Trumbore, triangle.rs:32-92, then accepts any
// t >= t_min, t > EPSILON) and its right one against the left's t when the left hit (else NaN). So
// the answer is a scan of the BVH's leaf objects in DFS order (lower.cpp bvh_emit's table), no box
// test at all: the same arithmetic per triangle, the same selection, as the literal recursion
// (oracle.c bvh_node_hit), which visited every node of C4's 20k-triangle tree from one lane (~20 ms a
// segment: the replay pass's tail after C4's fast kernel) where the scan's loads do not wait on each
// other.
template <uint32_t kF>
RT_DEV bool bvh_hit_nan_tmax(const DevScene& S, const f4* wrapper, const Ray& r, float tmin, float& closest,
                             uint32_t& hit_code) {
    const f4* T = S.nodes + (size_t)__float_as_uint(ld4c(wrapper + 7).y) * rtdev::kBvhNodeF4;
    const uint32_t n = __float_as_uint(ld1_at(T, 0u));
    const float nan = __uint_as_float(0x7fc00000u);
    bool any = false;
    float best = 0.0f;
    uint32_t best_code = 0u;
    auto test = [&](uint32_t i, float tmax, float& t) {
        const uint32_t idx = rtdev::leaf_index(__float_as_uint(ld1_at(T, 16u + 4u * i)));
        return tri_t(ld4(S.tri + 3 * (size_t)idx), ld4(S.tri + 3 * (size_t)idx + 1), ld4(S.tri + 3 * (size_t)idx + 2), r,
                     tmin, tmax, t);
    };
    for (uint32_t i = 0; i < n;) {
        const uint32_t e = __float_as_uint(ld1_at(T, 16u + 4u * i));
        const bool pair = (e & rtdev::kDfsPairLeft) != 0u && i + 1u < n;
        float tl = 0.0f, tr = 0.0f;
        const bool hl = test(i, nan, tl);
        const bool hr = pair && test(i + 1u, hl ? tl : nan, tr);
        // the leaf node's result: its right object when that hit (then tr <= tl), else its left one
        if (hl || hr) {
            const float t = hr ? tr : tl;
            if (!any || !(best < t)) {  // the tree's `l.t < r.t ? l : r`, the earlier nodes on the left
                any = true;
                best = t;
                best_code = __float_as_uint(ld1_at(T, 16u + 4u * (hr ? i + 1u : i))) & ~rtdev::kDfsPairLeft;
            }
        }
        i += pair ? 2u : 1u;
    }
    if (!any) return false;
    closest = best;
    hit_code = best_code;
    return true;
}

// RT_PEEL_WRAPPER: bvh_hit tests the wrapper's slot (the root box) before the traversal loop (0:
// the loop's first trip does, A/B).
#ifndef RT_PEEL_WRAPPER
#define RT_PEEL_WRAPPER 1
#endif
constexpr bool kPeelWrapper = RT_PEEL_WRAPPER;
template <int kKind, uint32_t kF = kFAll>
RT_DEV bool bvh_hit(const DevScene& S, float delta, uint32_t root, const Ray& r, float tmin, float& closest,
                    uint32_t& hit_code, uint32_t* stk, uint32_t mode, bool& replay) {
    PROF_T0(pcall);
    PROF_T0(psetup);
    const f4* wrapper = S.nodes + (size_t)root * rtdev::kBvhNodeF4;
    const V inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    if constexpr (kKind == 1 || kKind == 2) {
        const RayD q = to_d(r);
        const uint32_t w2 = __float_as_uint(ld4c(wrapper + 7).z);
        if constexpr (kKind == 2) {
            const uint32_t pid = __float_as_uint(S.nodes2[4 * (size_t)w2 + 3].z);
            if (pid) return bvh_hit_hrpp(S, w2, pid, r, q, inv, tmin, closest, hit_code, stk);
        }
        return bvh_hit_reference(S, w2, r, q, inv, tmin, closest, hit_code, stk);
    }
    // The fast traversal takes only the rays ray_route admits (a zero, denormal or non-finite
    // direction component would give 0 * inf = NaN slab values, which the packed child test, the
    // pruning margin and the empty slots' infinite boxes must not see, except in a triangle-only
    // BVH; e.g. H = 1 images divide by H - 1 = 0 in renderer.rs:141). A non-finite origin is
    // handed over too: a NaN rect hit leaves a NaN origin for the next bounce, which the replay
    // pass can meet after a bounce the fast kernel never traced. The reference kernel takes them.
    {
        const uint32_t route = ray_route<kKind, kF>(r, inv, closest, wrapper, mode);
        if (route == kRayNoHit) return false;
        if constexpr (kKind == 3) {
            if (route == kRayHandOver) {
                if constexpr ((kF & kFTri) != 0u) {
                    const bool fin = __builtin_fabsf(r.o.x) < kInf && __builtin_fabsf(r.o.y) < kInf &&
                                     __builtin_fabsf(r.o.z) < kInf && __builtin_fabsf(r.d.x) < kInf &&
                                     __builtin_fabsf(r.d.y) < kInf && __builtin_fabsf(r.d.z) < kInf;
                    if (closest != closest && fin &&
                        (__float_as_uint(ld4c(wrapper + 7).w) & rtdev::kBvhTriOnly) != 0u &&
                        !(kPruneAllExpBuild && (mode & kModePruneAllExp)))
                        return bvh_hit_nan_tmax<kF>(S, wrapper, r, tmin, closest, hit_code);
                }
                return bvh_hit_reference(S, __float_as_uint(ld4c(wrapper + 7).z), r, to_d(r), inv, tmin, closest, hit_code,
                                         stk);
            }
        }
        if (route == kRayHandOver) {
            replay = true;
            return false;
        }
    }
    PROF_ADD(kPrBvhSetup, psetup);
    Trav tv{root, 0u, 0u, closest, false, kNoNode};
    if constexpr (kPeelWrapper) {
        // The wrapper's one slot (the root's box, bvh.rs:370) tested outside the loop, from scalar
        // loads at the wave-uniform wrapper address: the loop's first trip, which loads the same
        // rows for every lane with vector loads, sorts four keys of which three are empty and
        // pushes nothing, becomes a handful of VALU operations, and a lane whose ray misses the
        // root box never enters the loop. The same interval, prune bound and result as
        // child_keys4_nf's slot 0 (see there; no NaN slab value under ray_route), then cur = the
        // root, with nothing on the stack: the state the loop's first trip leaves.
        const f4 w0 = ld4c(wrapper), w1 = ld4c(wrapper + 1), w2 = ld4c(wrapper + 2), w3 = ld4c(wrapper + 3),
                 w4 = ld4c(wrapper + 4), w5 = ld4c(wrapper + 5), w6 = ld4c(wrapper + 6), w7 = ld4c(wrapper + 7);
        const bool prune = (__float_as_uint(w7.w) & rtdev::kBvhPrunable) != 0u ||
                           (kPruneAllExpBuild && (mode & kModePruneAllExp));
        const float dmi = delta * fmaxf(fmaxf(__builtin_fabsf(inv.x), __builtin_fabsf(inv.y)), __builtin_fabsf(inv.z));
        const bool sx = inv.x < 0.0f, sy = inv.y < 0.0f, sz = inv.z < 0.0f;
        const float tnx = ((sx ? w3.x : w0.x) - r.o.x) * inv.x, tfx = ((sx ? w0.x : w3.x) - r.o.x) * inv.x;
        const float tny = ((sy ? w4.x : w1.x) - r.o.y) * inv.y, tfy = ((sy ? w1.x : w4.x) - r.o.y) * inv.y;
        const float tnz = ((sz ? w5.x : w2.x) - r.o.z) * inv.z, tfz = ((sz ? w2.x : w5.x) - r.o.z) * inv.z;
        const float lo = __builtin_fmaxf(__builtin_fmaxf(tnx, tny), __builtin_fmaxf(tnz, tmin));
        const float hi = __builtin_fminf(__builtin_fminf(tfx, tfy), __builtin_fminf(tfz, closest));
        const float te = lo - (prune ? dmi : 0.0f);
        if (lo <= hi && te <= (prune ? prune_bound(closest) : kInf)) {
            tv.cur = __float_as_uint(w6.x);
            bvh_run<kKind, kF, false>(S, delta, wrapper, r, inv, tmin, closest, hit_code, stk, mode, tv, 0u);
        }
    } else {
        bvh_run<kKind, kF, false>(S, delta, wrapper, r, inv, tmin, closest, hit_code, stk, mode, tv, 0u);
    }
    const bool any = tv.any;
    PROF_ADD(kPrBvhCall, pcall);
    trav_audit(S, wrapper, root, r, inv, tmin, tv, closest, hit_code, stk);
    return any;
}

// The fast BVH4 traversal loop from state tv: tv.cur is the next node to visit, tv.sp the
// entries on the lane's stack, tv.tmax_entry the t_max the BVH was entered with (every box
// test uses it), tv.best_rank / tv.any the best candidate so far (its t in `closest`, its
// code in `hit_code`). Returns true when the traversal is complete.
// kSusp (the suspending world walk, world_walk): before each visit, once the wave has made
// kSuspMinTrips visits in this call and at most `susp` of its lanes are still traversing,
// every remaining lane stops, keeps its state in tv (its stack stays in LDS) and returns
// false; the walk resumes it on a later trip of the sample loop, together with the lanes
// that reach the same BVH then. The visit order and every value are unchanged, only when a
// visit runs differs, so the result is the same bits.
#ifndef RT_POP_PREFETCH
#define RT_POP_PREFETCH 0
#endif
template <uint32_t kF>
constexpr bool kPopPrefetch = RT_POP_PREFETCH && (kF & (kFTri | kFDeep)) == 0u;
template <int kKind, uint32_t kF, bool kSusp>
RT_DEV bool bvh_run(const DevScene& S, float delta, const f4* wrapper, const Ray& r, V inv, float tmin, float& closest,
                    uint32_t& hit_code, uint32_t* stk, uint32_t mode, Trav& tv, uint32_t susp) {
    const float tmax_entry = tv.tmax_entry;
    const bool prune = (__float_as_uint(ld4c(wrapper + 7).w) & rtdev::kBvhPrunable) != 0u ||
                       (kPruneAllExpBuild && (mode & kModePruneAllExp));
    const float dmi = delta * fmaxf(fmaxf(__builtin_fabsf(inv.x), __builtin_fabsf(inv.y)), __builtin_fabsf(inv.z));
    const bool leaf_boxes = prune && !(mode & kModeNoLeafBoxes);
    // Byte offsets of each axis's near-plane row in a node (min.a rows 0-2, max.a rows 3-5;
    // the max plane is entered first when 1/d < 0); the far row is the other one (off ^ c).
    [[maybe_unused]] const uint32_t hnx = inv.x < 0.0f ? 48u : 0u, hny = inv.y < 0.0f ? 64u : 16u,
                                    hnz = inv.z < 0.0f ? 80u : 32u;
    bool any = tv.any;
    uint32_t best_rank = tv.best_rank, sp = tv.sp, cur = tv.cur, pend = tv.pend;
    // Leaf postponement (the triangle preset; q = RT_LEAF_Q sixteenths, RT_OPT_TUNE bits 24-27
    // override it for A/B, 15 = off): a lane that reaches a leaf node parks it in `pend` and goes
    // on with the next node of its stack; the wave tests the parked leaves together once at least
    // q/16 of its traversing lanes hold one, or when no lane can advance otherwise. The leaf test
    // ran at a few lanes per execution when every lane tested its leaf at once. Every candidate
    // still meets the same tests and merges into (closest, DFS rank) by the same order-independent
    // rule, and pruning stays conservative with a later `closest`, so the result is the same bits;
    // only the visit order changes. Measured (same box, bit-identical, 50-spp C4 frames): 1061 ->
    // 1094 Msamples/s at q = 8 (q = 4: 1093, 6: 1097, 10: 1080); on the sphere presets, where a
    // leaf hit prunes the rest of the stack, no q beat testing at once (runtime-q build: C3 q = 8
    // -1.4%, C1 -3%), so they compile the immediate loop, instruction for instruction the old one
    // (profiles/r04/experiments/leaf_postpone_*.log).
    constexpr bool kPostpone = (kF & kFTri) != 0u && kKind == 0;
    const uint32_t tq = (mode >> 24) & 15u;
    const uint32_t lq = !kPostpone ? 0u : (tq == 15u ? 0u : (tq ? tq : (uint32_t)RT_LEAF_Q));
    bool finished = true;
    [[maybe_unused]] uint32_t trips = 0;
#ifdef RT_PROFILE_REGIONS
    uint32_t visits = 0;
#endif
    for (;;) {
        if constexpr (kSusp) {
            if (trips >= kSuspMinTrips && (uint32_t)__popcll(__ballot(1)) <= susp) {
                finished = false;
                break;
            }
            ++trips;
        }
        // this trip: test one leaf node (the parked one first), or park the current leaf, or
        // visit the current interior node. Without postponement `cur` is always a node here.
        uint32_t lnode = kNoNode;
        bool popnext = false, do_int;
        if constexpr (kPostpone) {
            const bool cur_leaf = cur != kNoNode && (cur & rtdev::kLeafNodeFlag) != 0u;
            const bool has_pend = pend != kNoNode;
            bool leafphase = true;
            if (lq) {
                const bool can_adv = cur != kNoNode && (!cur_leaf || !has_pend);
                const uint32_t n_act = (uint32_t)__popcll(__ballot(1)), n_pend = (uint32_t)__popcll(__ballot(has_pend));
                leafphase = __ballot(can_adv) == 0ull || n_pend * 16u >= lq * n_act;
            }
            if (leafphase) {
                if (has_pend) {
                    lnode = pend;
                    pend = kNoNode;
                } else if (cur_leaf) {
                    lnode = cur;
                    popnext = true;
                }
            } else if (cur_leaf && !has_pend) {
                pend = cur;
                popnext = true;
            }
            do_int = lnode == kNoNode && !popnext && cur != kNoNode && !cur_leaf;
        } else {
            const bool cur_leaf = (cur & rtdev::kLeafNodeFlag) != 0u;
            lnode = cur_leaf ? cur : kNoNode;
            do_int = !cur_leaf;
        }
        // The near-plane row offsets. The sphere-BVH presets rederive them each trip from the
        // direction's sign bits (volatile asm is not hoisted: three loop-invariant offsets live
        // across the loop, where registers are scarcest, pushed C3's sample-loop state into
        // scratch, 1.7% slower); the triangle preset keeps them hoisted (2.3% faster there).
        uint32_t onx, ony, onz;
        if constexpr ((kF & kFTri) != 0u) {
            onx = hnx;
            ony = hny;
            onz = hnz;
        } else {
            uint32_t msx, msy, msz;  // 0 or ~0: 1/d < 0 on the axis
            asm volatile("v_ashrrev_i32 %0, 31, %1" : "=v"(msx) : "v"(inv.x));
            asm volatile("v_ashrrev_i32 %0, 31, %1" : "=v"(msy) : "v"(inv.y));
            asm volatile("v_ashrrev_i32 %0, 31, %1" : "=v"(msz) : "v"(inv.z));
            onx = msx & 48u;
            ony = (msy & 48u) + 16u;
            onz = (msz & 48u) + 32u;
        }
#ifdef RT_LEAF_AUDIT
        {
            const uint32_t vis = lnode != kNoNode ? lnode : cur;
            if ((vis != kNoNode && (vis & ~rtdev::kLeafNodeFlag) >= S.num_nodes) || sp > S.stack_depth + S.spill_depth) {
                atomicAdd(&g_bounds_audit_count, 1u);
                break;
            }
        }
#endif
#ifdef RT_PROFILE_REGIONS
        ++visits;
#endif
        // RT_POP_PREFETCH (A/B): the stack top read at the start of the trip, beside the node loads. A trip
        // that pops has pushed nothing, so the first entry its pop loop takes is this one.
        [[maybe_unused]] uint32_t pf_node = 0u;
        [[maybe_unused]] float pf_t = 0.0f;
        if constexpr (kPopPrefetch<kF>) {
            const uint32_t top = (sp > 0u ? sp - 1u : 0u) * 128u;
            pf_node = stk[top];
            pf_t = __uint_as_float(stk[top + 64u]);
        }
        PROF_T0(pt);
        if (lnode != kNoNode) {
            // The 1-2 leaf children of ONE reference BVH2 node, left then right,
            // and that node's result formed exactly like bvh.rs:377-414: the left
            // leaf is tested with the BVH's entry t_max, the right one with the
            // left hit's t (t_max_for_right), and `if left.t < right.t {left} else
            // {right}`. This matters for f64 spheres: sphere.rs compares its root
            // against the f32 t_max before rounding t to f32, so a sphere whose
            // rounded t equals another candidate's passes or fails depending on
            // which t_max it saw. The node result then joins (closest, DFS rank)
            // like the tree-min does.
            const uint32_t nbo = (lnode & ~rtdev::kLeafNodeFlag) * (rtdev::kBvhNodeF4 * 16u);  // node byte offset
            const f4* nd = S.nodes;
            const float2 nx2 = ld2_at(nd, nbo + onx), ny2 = ld2_at(nd, nbo + ony), nz2 = ld2_at(nd, nbo + onz),
                         fx2 = ld2_at(nd, nbo + (onx ^ 48u)), fy2 = ld2_at(nd, nbo + (ony ^ 80u)),
                         fz2 = ld2_at(nd, nbo + (onz ^ 112u)), chs = ld2_at(nd, nbo + 96u), rks = ld2_at(nd, nbo + 112u);
            float tmr = tmax_entry, nt = 0.0f;
            bool nh = false;
            uint32_t ncode = 0u, nrank = 0u;
            const uint32_t nleaf = __float_as_uint(chs.y) == rtdev::kChildEmpty ? 1u : 2u;
            float llo[2] = {-kInf, -kInf}, lhi[2] = {kInf, kInf};
            if (leaf_boxes) leaf_intervals2_nf(nx2, ny2, nz2, fx2, fy2, fz2, r, inv, delta, llo, lhi);
            for (uint32_t k = 0; k < nleaf; ++k) {
                const uint32_t lcode = __float_as_uint(k ? chs.y : chs.x), rank = __float_as_uint(k ? rks.y : rks.x);
#ifdef RT_LEAF_AUDIT
                const float2 bx0 = ld2(S.nodes + nbo / 16u, 0), by0 = ld2(S.nodes + nbo / 16u, 1),
                             bz0 = ld2(S.nodes + nbo / 16u, 2), bx1 = ld2(S.nodes + nbo / 16u, 3),
                             by1 = ld2(S.nodes + nbo / 16u, 4), bz1 = ld2(S.nodes + nbo / 16u, 5);
                const float x0 = k ? bx0.y : bx0.x, y0 = k ? by0.y : by0.x, z0 = k ? bz0.y : bz0.x;
                const float x1 = k ? bx1.y : bx1.x, y1 = k ? by1.y : by1.x, z1 = k ? bz1.y : bz1.x;
#endif
                // the right leaf can only matter if t <= min(closest, left t)
                const float bound = tmr < closest ? tmr : closest;
                if (!leaf_boxes || leaf_interval_may_hit(k ? llo[1] : llo[0], k ? lhi[1] : lhi[0], tmin, bound)) {
                    PROF_T0(pl);
                    // Only candidates whose f32 t can tie or beat closest matter, so
                    // the test may use min(t_max, nextup(closest)): a root in
                    // (closest, nextup] is still judged against the reference's own
                    // t_max, anything beyond rounds above closest and loses anyway.
                    const float cap = closest < kInf ? __uint_as_float(__float_as_uint(closest) + 1u) : kInf;
                    float c = tmr < cap ? tmr : cap;
                    uint32_t code = 0u;
                    const RayD q = to_d(r);  // f64 ray for sphere leaves, rebuilt here rather than kept live
                    ABLATE(kAbLeaf2, float c2 = c; uint32_t h2 = 0u;
                           if (leaf_hit<kF>(S, lcode, r, q, tmin, c2, h2) && h2 == 0x7fffffffu) c = -1.0f;);
                    // cube sides from the ray's reciprocals (side_t_rcp) except in the triangle preset,
                    // whose instance lost 1.6% to the extra code (C3 +2%; uniform_entries_ab.log)
                    bool hit;
                    if constexpr (kLeafEmbed<kF>) {
                        const uint32_t ltype = rtdev::leaf_type(lcode);
                        // leaf k's lane of rows 0-6 (the node's line, just fetched; the address needs
                        // no record index, so the loads do not wait on the child row)
                        const uint32_t lo = nbo + 4u * k;
                        if (ltype == rtdev::kLeafSphere) {  // (cx, cy, cz, r) in lane 2 + k of rows 0, 1, 2, 6
                            const f4 sp{ld1_at(nd, lo + 8u), ld1_at(nd, lo + 24u), ld1_at(nd, lo + 40u), ld1_at(nd, lo + 104u)};
                            float ts;
                            hit = sphere_t(sp, q, tmin, c, ts);
                            if (hit) {
                                c = ts;
                                code = lcode;
                            }
                        } else if (ltype == rtdev::kLeafCube) {  // its leaf box (lane k of rows 0-5) is its bounds
                            hit = cube_hit<(kF & kFTri) == 0u>(S, rtdev::leaf_index(lcode), ld1_at(nd, lo), ld1_at(nd, lo + 16u),
                                                               ld1_at(nd, lo + 32u), ld1_at(nd, lo + 48u), ld1_at(nd, lo + 64u),
                                                               ld1_at(nd, lo + 80u), r, inv, tmin, c, code);
                        } else {
                            hit = leaf_hit<kF, (kF & kFTri) == 0u, false, true>(S, lcode, r, q, tmin, c, code, inv);
                        }
                    } else {
                        hit = leaf_hit<kF, (kF & kFTri) == 0u>(S, lcode, r, q, tmin, c, code, inv);
                    }
                    if (hit) {
                        // cube faces rank + 0..5 (the face leaf_hit's list walk kept)
                        const uint32_t rk = rank + (rtdev::leaf_type(lcode) == rtdev::kLeafCube
                                                        ? rtdev::leaf_index(code) - rtdev::leaf_index(lcode)
                                                        : 0u);
                        if (!nh || !(nt < c)) {
                            nh = true;
                            nt = c;
                            ncode = code;
                            nrank = rk;
                        }
                        tmr = c;
                    }
                    PROF_ADD(kPrLeafTest, pl);
                } else {
                    LEAF_AUDIT(lcode, rank, x0, y0, z0, x1, y1, z1);
                }
            }
            if (nh && (nt < closest || (nt == closest && nrank > best_rank))) {
                closest = nt;
                best_rank = nrank;
                hit_code = ncode;
                any = true;
            }
        }
        float t0 = kInf, t1 = kInf, t2 = kInf, t3 = kInf;
        uint32_t c0 = rtdev::kChildEmpty, c1 = rtdev::kChildEmpty, c2 = rtdev::kChildEmpty, c3 = rtdev::kChildEmpty;
        if (do_int) {
            // interior slots: reference box test, prune bound, nearest first
            const uint32_t nbo = cur * (rtdev::kBvhNodeF4 * 16u);  // node byte offset
            const f4* nd = S.nodes;
            const f4 nx = ld4_at(nd, nbo + onx), ny = ld4_at(nd, nbo + ony), nz = ld4_at(nd, nbo + onz),
                     fx = ld4_at(nd, nbo + (onx ^ 48u)), fy = ld4_at(nd, nbo + (ony ^ 80u)),
                     fz = ld4_at(nd, nbo + (onz ^ 112u)), chf = ld4_at(nd, nbo + 96u);
            c0 = __float_as_uint(chf.x);
            c1 = __float_as_uint(chf.y);
            c2 = __float_as_uint(chf.z);
            c3 = __float_as_uint(chf.w);
            ABLATE(kAbKeys2, const f4 mnx = inv.x < 0.0f ? fx : nx; const f4 mxx = inv.x < 0.0f ? nx : fx;
                   const f4 mny = inv.y < 0.0f ? fy : ny; const f4 mxy = inv.y < 0.0f ? ny : fy;
                   const f4 mnz = inv.z < 0.0f ? fz : nz; const f4 mxz = inv.z < 0.0f ? nz : fz;
                   float k2 = child_key(mnx.x, mny.x, mnz.x, mxx.x, mxy.x, mxz.x, r, inv, tmin, tmax_entry,
                                                  closest, prune, dmi) +
                                        child_key(mnx.y, mny.y, mnz.y, mxx.y, mxy.y, mxz.y, r, inv, tmin, tmax_entry,
                                                  closest, prune, dmi) +
                                        child_key(mnx.z, mny.z, mnz.z, mxx.z, mxy.z, mxz.z, r, inv, tmin, tmax_entry,
                                                  closest, prune, dmi) +
                                        child_key(mnx.w, mny.w, mnz.w, mxx.w, mxy.w, mxz.w, r, inv, tmin, tmax_entry,
                                                  closest, prune, dmi);
                   if (k2 == -1.0f) c0 = 0u;);
            float key[4];
            child_keys4_nf(nx, ny, nz, fx, fy, fz, r, inv, tmin, tmax_entry, prune ? prune_bound(closest) : kInf,
                           prune ? dmi : 0.0f, key);
            t0 = key[0];
            t1 = key[1];
            t2 = key[2];
            t3 = key[3];
        }
        PROF_ADD(kPrBvhTrip, pt);
        PROF_T0(pp);
        // LDS stack; with kFDeep the entries past stack_depth go to the HBM spill area
        auto push = [&](uint32_t node, float t) {
            if (!(kF & kFDeep) || sp < S.stack_depth) {
                stk[sp * 128u] = node;
                stk[sp * 128u + 64u] = __float_as_uint(t);
            } else {
                uint32_t* g = S.stack_spill +
                              (((size_t)blockIdx.x * S.spill_depth + (sp - S.stack_depth)) * 64u + threadIdx.x) * 2u;
                g[0] = node;
                g[1] = __float_as_uint(t);
            }
            sp += 1u;
        };
        sort2(t0, c0, t1, c1);
        sort2(t2, c2, t3, c3);
        sort2(t0, c0, t2, c2);
        sort2(t1, c1, t3, c3);
        sort2(t1, c1, t2, c2);
        if (t0 != kInf) {  // visit the nearest next, push the others far to near
            if (t3 != kInf) push(c3, t3);
            if (t2 != kInf) push(c2, t2);
            if (t1 != kInf) push(c1, t1);
            cur = c0;
            if constexpr (!kPostpone) {
                PROF_ADD(kPrBvhPush, pp);
                continue;
            }
        } else if (!kPostpone || do_int) {
            popnext = true;
        }
        PROF_ADD(kPrBvhPush, pp);
        PROF_T0(ppop);
        if (popnext) {
            bool found = false;
            [[maybe_unused]] bool first = true;
            while (sp > 0u) {
                sp -= 1u;
                uint32_t cand;
                float tenter;
                if (kPopPrefetch<kF> && first) {
                    cand = pf_node;
                    tenter = pf_t;
                    first = false;
                } else if (!(kF & kFDeep) || sp < S.stack_depth) {
                    cand = stk[sp * 128u];
                    tenter = __uint_as_float(stk[sp * 128u + 64u]);
                } else {
                    const uint32_t* g = S.stack_spill +
                                        (((size_t)blockIdx.x * S.spill_depth + (sp - S.stack_depth)) * 64u + threadIdx.x) * 2u;
                    cand = g[0];
                    tenter = __uint_as_float(g[1]);
                }
                if (!prune || !(tenter > prune_bound(closest))) {
                    cur = cand;
                    found = true;
                    break;
                }
            }
            if (!found) {
                if constexpr (!kPostpone) {
                    PROF_ADD(kPrBvhPop, ppop);
                    break;
                } else {
                    cur = kNoNode;
                }
            }
        }
        PROF_ADD(kPrBvhPop, ppop);
        if constexpr (kPostpone) {
            if (cur == kNoNode && pend == kNoNode) break;
        }
    }
    tv = Trav{cur, sp, best_rank, tmax_entry, any, pend};
#ifdef RT_PROFILE_REGIONS
    {
        const uint32_t b = trips_bin(visits);
        uint32_t m = visits;
        for (int off = 32; off > 0; off >>= 1) {
            uint32_t o = __shfl_xor(m, off);
            m = o > m ? o : m;
        }
        const uint32_t first = (uint32_t)__builtin_ctzll(__ballot(1));
        for (uint32_t bin = 0; bin < 8u; ++bin) {
            const uint32_t n = (uint32_t)__popcll(__ballot(b == bin));
            if (__lane_id() == first && n) prof_lds[3u * kPrCount + bin] += n;
        }
        if (__lane_id() == first) prof_lds[3u * kPrCount + 8u + trips_bin(m)] += 1u;
    }
#endif
    return finished;
}

// Translate (instance.rs:39) / RotateY (instance.rs:104-110, 121-124) applied to a ray.
RT_DEV Ray apply_op(f4 op, Ray r) {
    if (op.w == 0.0f) {
        r.o = r.o - xyz(op);
    } else {
        float s = op.x, c = op.y;
        r.o = mk(c * r.o.x - s * r.o.z, r.o.y, s * r.o.x + c * r.o.z);
        r.d = mk(c * r.d.x - s * r.d.z, r.d.y, s * r.d.x + c * r.d.z);
    }
    return r;
}

// sphere_surely_missed for two spheres at once (v_pk_mul_f32 / v_pk_add_f32: the
// same rounded operations per element; the bound holds for any evaluation order).
RT_DEV void spheres_surely_missed2(f4 s0, f4 s1, const Ray& r, float a, bool& m0, bool& m1) {
    const pk2 ocx = pk(r.o.x, r.o.x) - pk(s0.x, s1.x), ocy = pk(r.o.y, r.o.y) - pk(s0.y, s1.y),
              ocz = pk(r.o.z, r.o.z) - pk(s0.z, s1.z);
    const pk2 dx = pk(r.d.x, r.d.x), dy = pk(r.d.y, r.d.y), dz = pk(r.d.z, r.d.z), a2 = pk(a, a);
    const pk2 hb = (ocx * dx + ocy * dy) + ocz * dz;
    const pk2 oc2 = (ocx * ocx + ocy * ocy) + ocz * ocz;
    const pk2 rad = pk(s0.w, s1.w);
    const pk2 r2 = rad * rad;
    const pk2 hb2 = hb * hb;
    const pk2 disc = hb2 - a2 * (oc2 - r2);
    const pk2 m = hb2 + a2 * (oc2 + r2);
    const pk2 lim = pk(-0x1p-16f, -0x1p-16f) * m;
    m0 = m[0] > 0x1p-100f && disc[0] < lim[0];
    m1 = m[1] > 0x1p-100f && disc[1] < lim[1];
}

// A top-level entry's record is the same for every lane of the wave (the list walk is a wave-uniform
// loop). In the triangle-BVH and flat-list presets its fields are read once into scalar registers
// (readfirstlane), so the wave branches on them instead of masking lanes, and a top-level rectangle's
// plane axis picks one of three code paths instead of every lane selecting the ray components per
// axis. Measured (same box, bit-identical, profiles/r05/experiments/uniform_entries_ab.log): C4 +3.5%,
// C5 +0.8%; C3 -1% and C2 -4% (register allocation), so their presets keep the vector reads.
template <uint32_t kF>
constexpr bool kUniformEntries = (kF & kFTri) != 0u || (kF & (kFBvh | kFRuns)) == 0u;
template <uint32_t kF>
RT_DEV uint32_t uni(uint32_t v) {
    if constexpr (kUniformEntries<kF>) return __builtin_amdgcn_readfirstlane(v);
    return v;
}
// apply_op for a wave-uniform transform record: the Translate / RotateY choice is a scalar branch.
template <uint32_t kF>
RT_DEV Ray apply_op_u(f4 op, Ray r) {
    if (__uint_as_float(uni<kF>(__float_as_uint(op.w))) == 0.0f) {
        r.o = r.o - xyz(op);
    } else {
        float s = op.x, c = op.y;
        r.o = mk(c * r.o.x - s * r.o.z, r.o.y, s * r.o.x + c * r.o.z);
        r.d = mk(c * r.d.x - s * r.d.z, r.d.y, s * r.d.x + c * r.d.z);
    }
    return r;
}
constexpr uint32_t kRunPretestMin = 8u;  // sphere runs at least this long take the f32 pretest
// A GEOM or BVH entry (the caller guarantees E is wave-uniform). Only instances
// with kFRuns carry the f32 pretest of long sphere runs, only those with kFBvh the
// BVH traversal (the host launches an instance whose features cover the scene's).
template <int kKind, uint32_t kF>
RT_DEV bool entry_geom_hit(const DevScene& S, float delta, const DevEntry* E, Ray r, float tmin, float& closest,
                           uint32_t& hit_code, uint32_t* stk, uint32_t mode, bool& replay) {
    uint32_t ntf = uni<kF>(cst(E)->ntf);
    for (uint32_t i = 0; i < ntf; ++i) r = apply_op_u<kF>(ld4c(&E->tf[i]), r);
    const uint32_t kind = uni<kF>(cst(E)->kind);
    if (kind == rtdev::kEntSphereRun) {  // consecutive top-level spheres, in list order
        const uint32_t first = uni<kF>(cst(E)->payload), n = uni<kF>(cst(E)->pad[0]);
        const RayD q = to_d(r);
        const bool pretest = (kF & kFRuns) && n >= kRunPretestMin && !(mode & kModeNoPretest);  // long lists (random_spheres without a BVH): most spheres are misses
        bool any = false;
        auto test = [&](uint32_t i, f4 sp, bool missed) {  // sphere i in list order (hittable.rs:110-116)
            float t;
            if (missed) {
#ifdef RT_LEAF_AUDIT
                if (sphere_roots(sp, q).ok) atomicAdd(&g_audit_count, 1u);  // audit: the f64 test must reject too
#endif
                return;
            }
            if (sphere_t(sp, q, tmin, closest, t)) {
                closest = t;
                hit_code = rtdev::leaf_code(rtdev::kLeafSphere, first + i);
                any = true;
            }
        };
        uint32_t i = 0;
        if (pretest) {
            const float a = (r.d.x * r.d.x + r.d.y * r.d.y) + r.d.z * r.d.z;
            for (; i + 1u < n; i += 2u) {  // pairs: one packed pretest, then each sphere in order
                const f4 s0 = ld4c(S.sph + first + i), s1 = ld4c(S.sph + first + i + 1u);
                bool m0, m1;
                spheres_surely_missed2(s0, s1, r, a, m0, m1);
                test(i, s0, m0);
                test(i + 1u, s1, m1);
            }
        }
        for (; i < n; ++i) {
            const f4 sp = ld4c(S.sph + first + i);
            test(i, sp, pretest && sphere_surely_missed(sp, r));
        }
        return any;
    }
    if (kind == rtdev::kEntRectRun) {  // consecutive untransformed top-level rectangles, in list order
        const uint32_t first = uni<kF>(cst(E)->payload), n = uni<kF>(cst(E)->pad[0]);
        bool any = false;
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t idx = first + i;
            const f4 r0 = ld4c(S.rect + 2 * idx), r1 = ld4c(S.rect + 2 * idx + 1);
            float t;
            bool h;
            if constexpr (kUniformEntries<kF>) {  // the plane axis is the wave's (a scalar branch)
                const uint32_t axis = __builtin_amdgcn_readfirstlane(__float_as_uint(r1.y));
                if (axis == 0u)  // XY: plane z
                    h = side_t(r0.x, r.o.z, r.d.z, r.o.x, r.d.x, r.o.y, r.d.y, r0.y, r0.z, r0.w, r1.x, tmin, closest, t);
                else if (axis == 1u)  // XZ: plane y
                    h = side_t(r0.x, r.o.y, r.d.y, r.o.x, r.d.x, r.o.z, r.d.z, r0.y, r0.z, r0.w, r1.x, tmin, closest, t);
                else  // YZ: plane x
                    h = side_t(r0.x, r.o.x, r.d.x, r.o.y, r.d.y, r.o.z, r.d.z, r0.y, r0.z, r0.w, r1.x, tmin, closest, t);
            } else {
                h = rect_t(r0, r1, r, tmin, closest, t);
            }
            if (h) {
                closest = t;
                hit_code = rtdev::leaf_code(rtdev::kLeafRect, idx);
                any = true;
            }
        }
        return any;
    }
    if (kind == rtdev::kEntBvh) {
        if constexpr ((kF & kFBvh) == 0u) {
            return false;  // not reached: the scene has no BVH
        } else {
            ABLATE(kAbBvh2, float c2 = closest; uint32_t h2 = 0u; bool rp = false;
                   if (bvh_hit<kKind, kF>(S, delta, cst(E)->payload, r, tmin, c2, h2, stk, mode, rp) && h2 == 0x7fffffffu)
                       closest = -1.0f;);
            return bvh_hit<kKind, kF>(S, delta, uni<kF>(cst(E)->payload), r, tmin, closest, hit_code, stk, mode,
                                            replay);
        }
    }
    if constexpr (kUniformEntries<kF>) {
        // A top-level rectangle (walls, lights): its record is the same for the whole wave, so its
        // plane axis is read once (readfirstlane) and the wave branches on it, instead of every lane
        // selecting the six ray components per axis (rect_axes). Same operations as rect_t.
        const uint32_t code = __builtin_amdgcn_readfirstlane(cst(E)->payload);
        if (rtdev::leaf_type(code) == rtdev::kLeafRect) {
            const uint32_t idx = rtdev::leaf_index(code);
            const f4 r0 = ld4c(S.rect + 2 * idx), r1 = ld4c(S.rect + 2 * idx + 1);
            const uint32_t axis = __builtin_amdgcn_readfirstlane(__float_as_uint(r1.y));
            float t;
            bool h;
            if (axis == 0u)  // XY: plane z
                h = side_t(r0.x, r.o.z, r.d.z, r.o.x, r.d.x, r.o.y, r.d.y, r0.y, r0.z, r0.w, r1.x, tmin, closest, t);
            else if (axis == 1u)  // XZ: plane y
                h = side_t(r0.x, r.o.y, r.d.y, r.o.x, r.d.x, r.o.z, r.d.z, r0.y, r0.z, r0.w, r1.x, tmin, closest, t);
            else  // YZ: plane x
                h = side_t(r0.x, r.o.x, r.d.x, r.o.y, r.d.y, r.o.z, r.d.z, r0.y, r0.z, r0.w, r1.x, tmin, closest, t);
            if (h) {
                closest = t;
                hit_code = code;
            }
            return h;
        }
    }
    RayD q = to_d(r);
    ABLATE(kAbGeom2, float c2 = closest; uint32_t h2 = 0u;
           if (leaf_hit<kF | kFLeafRM>(S, cst(E)->payload, r, q, tmin, c2, h2) && h2 == 0x7fffffffu) closest = -1.0f;);
    return leaf_hit<kF | kFLeafRM, false, true>(S, uni<kF>(cst(E)->payload), r, q, tmin, closest, hit_code);  // top level: any primitive
}

// Medium-first bound (world_hit, fast kernel; DESIGN.md §4 "medium-first bound"). The first
// top-level ConstantMedium (S.mb_entry, sphere boundary) draws its ln(U) from the stream state the
// walk starts with, since no entry before it draws. Its scatter point is estimated here in f32 from
// a peeked draw; world_hit walks the entries before it with t_max = B (a little beyond the estimate
// C) instead of inf. Any hit <= C of those entries is then found with the same record (a box the
// reference test rejects at B holds no candidate <= C: the exact-pruning margin of bvh_hit), and if
// none is found the medium, entered with t_max = inf, scatters where the reference's would with any
// closest_so_far >= C — which medium_hit checks on the exact values (vbound), handing the sample to
// the reference kernel otherwise. kInf: no bound (no such medium, the ray misses its sphere or
// leaves it unscattered by the estimate).
#ifndef RT_MEDIUM_FIRST
#define RT_MEDIUM_FIRST 1
#endif
// Compiled into the sphere-BVH preset with marble textures (the book-2 final scene's, C3): same box,
// same bits, C3 93.4 -> 88.9 ms per 100-spp frame and one rank of 8 60.1 -> 57.2 ms; the BVH-only
// preset (C1, whose scenes have no media) does without its registers
// (profiles/r05/experiments/medium_first_ab.log).
template <uint32_t kF>
constexpr bool kMediumFirst = RT_MEDIUM_FIRST && (kF & kFBvh) != 0u && (kF & kFMarble) != 0u && (kF & kFTri) == 0u;
template <uint32_t kF>
RT_DEV float medium_first_estimate(const DevScene& S, const DevEntry* E, Ray r, const Rng& g, const Key& k) {
    const uint32_t ntf = cst(E)->ntf;
    for (uint32_t i = 0; i < ntf; ++i) r = apply_op_u<kF>(ld4c(&E->tf[i]), r);
    const DevEntry* B = S.entries + cst(E)->payload;
    Ray rb = r;
    const uint32_t bn = cst(B)->ntf;
    for (uint32_t i = 0; i < bn; ++i) rb = apply_op_u<kF>(ld4c(&B->tf[i]), rb);
    const f4 s = ld4c(S.sph + rtdev::leaf_index(cst(B)->payload));
    const V oc = rb.o - xyz(s);
    const float a = dot(rb.d, rb.d), hb = dot(oc, rb.d), cq = dot(oc, oc) - s.w * s.w;
    const float disc = hb * hb - a * cq;
    if (!(disc >= 0.0f)) return kInf;
    const float sq = __builtin_sqrtf(disc);
    const float r2 = (sq - hb) / a;
    float t1 = (-hb - sq) / a;
    if (t1 < 0.001f) t1 = 0.001f;
    if (!(t1 < r2)) return kInf;
    const float len = length(r.d);
    Rng p = g;  // the draw medium_hit will make, not consumed here
    const float hd = cst(E)->neg_inv_density * __logf(std01(p, k));
    if (!(hd < (r2 - t1) * len * (1.0f - 0x1p-10f))) return kInf;  // leaves (or about to): no bound
    return (t1 + hd / len) * (1.0f + 0x1p-8f) + 0x1p-16f;
}

// ConstantMedium::hit (hittable.rs:176-233); draws one U(0,1) once the clamped
// interval is non-empty, exactly where the reference does. vbound < inf: world_hit's medium-first
// bound C (above) with t_max = inf here; the hit must be the one every closest_so_far >= C gives.
template <int kKind, uint32_t kF>
RT_DEV bool medium_hit(const DevScene& S, float delta, const DevEntry* E, Ray r, float tmin, float tmax, Rng& g,
                       const Key& k, float& t_out, uint32_t* stk, uint32_t mode, bool& replay,
                       float vbound = kInf) {
    uint32_t ntf = uni<kF>(cst(E)->ntf);
    for (uint32_t i = 0; i < ntf; ++i) r = apply_op_u<kF>(ld4c(&E->tf[i]), r);
    const DevEntry* B = S.entries + uni<kF>(cst(E)->payload);
    float t1 = kInf, t2 = kInf;
    const uint32_t bkind = uni<kF>(cst(B)->kind), bcode = uni<kF>(cst(B)->payload);
    if (bkind == rtdev::kEntGeom && rtdev::leaf_type(bcode) == rtdev::kLeafSphere) {
        // boundary.hit(-inf, inf) then boundary.hit(t1 + 1e-4, inf) on one sphere:
        // the same two roots, selected against two intervals.
        Ray rb = r;
        uint32_t bn = uni<kF>(cst(B)->ntf);
        for (uint32_t i = 0; i < bn; ++i) rb = apply_op_u<kF>(ld4c(&B->tf[i]), rb);
        Roots R = sphere_roots(ld4c(S.sph + rtdev::leaf_index(bcode)), to_d(rb));
        ABLATE(kAbMedium2, Roots R2 = sphere_roots(ld4(S.sph + rtdev::leaf_index(cst(B)->payload)), to_d(rb));
               if (R2.r1 == -1.0) t1 = -1.0f;);
        if (!sphere_select(R, -kInf, kInf, t1)) return false;
        if (!sphere_select(R, t1 + 0.0001f, kInf, t2)) return false;
    } else if ((kF & kFTri) == 0u && bkind == rtdev::kEntGeom && rtdev::leaf_type(bcode) == rtdev::kLeafCube) {
        // boundary.hit twice on one Cube (cube.rs:84-93, six sides in list order): each
        // side's t = (k - o) / d and its in-rectangle test do not depend on the interval,
        // so they are computed once and both calls replay the list's selection on them,
        // NaN comparisons included (C5's smoke boxes: 138.8 -> 126.3 ms per 200-spp frame,
        // same bits). Left out of the triangle preset, whose scenes have no cube media and
        // whose register allocation the unused code cost 2.7% (C4).
        Ray rb = r;
        uint32_t bn = uni<kF>(cst(B)->ntf);
        for (uint32_t i = 0; i < bn; ++i) rb = apply_op_u<kF>(ld4c(&B->tf[i]), rb);
        const uint32_t idx = rtdev::leaf_index(bcode);
        const f4 s0 = ld4c(S.rect + 2 * idx);
        const float y1 = ld4c(S.rect + 2 * idx + 1).x, z1 = ld4c(S.rect + 2 * idx + 5).x;
        const float x0 = s0.y, x1 = s0.z, y0 = s0.w, z0 = s0.x;
        const float ox = rb.o.x, oy = rb.o.y, oz = rb.o.z, dx = rb.d.x, dy = rb.d.y, dz = rb.d.z;
        float tt[6];
        uint32_t in = 0u;  // bit f: side f's point lies inside its rectangle (rectangle.rs:36-65)
        {
            // (the six quotients from three reciprocals, div_rn, measured C5 -6%: kept as divisions;
            // profiles/r05/experiments/uniform_entries_ab.log)
            const float num[6] = {z0 - oz, z1 - oz, y0 - oy, y1 - oy, x0 - ox, x1 - ox};
            const float den[6] = {dz, dz, dy, dy, dx, dx};
#pragma unroll
            for (int f = 0; f < 6; ++f) tt[f] = num[f] / den[f];
        }
        auto side = [&](int f, float oa, float da, float ob, float db, float a0, float a1, float b0, float b1) {
            const float x = oa + tt[f] * da, y = ob + tt[f] * db;
            if (!(x < a0 || x > a1 || y < b0 || y > b1)) in |= 1u << f;
        };
        side(0, ox, dx, oy, dy, x0, x1, y0, y1);
        side(1, ox, dx, oy, dy, x0, x1, y0, y1);
        side(2, ox, dx, oz, dz, x0, x1, z0, z1);
        side(3, ox, dx, oz, dz, x0, x1, z0, z1);
        side(4, oy, dy, oz, dz, y0, y1, z0, z1);
        side(5, oy, dy, oz, dz, y0, y1, z0, z1);
        auto pick = [&](float lo, float& closest) {  // the HittableList walk: closest narrows
            bool any = false;
#pragma unroll
            for (int f = 0; f < 6; ++f)
                if (((in >> f) & 1u) && !(tt[f] < lo || tt[f] > closest)) {
                    closest = tt[f];
                    any = true;
                }
            return any;
        };
        if (!pick(-kInf, t1)) return false;
        if (!pick(t1 + 0.0001f, t2)) return false;
    } else {
        uint32_t dummy;
        if (!entry_geom_hit<kKind, kF>(S, delta, B, r, -kInf, t1, dummy, stk, mode, replay)) return false;
        if (!entry_geom_hit<kKind, kF>(S, delta, B, r, t1 + 0.0001f, t2, dummy, stk, mode, replay)) return false;
    }
    if (t1 < tmin) t1 = tmin;
    if (t2 > tmax) t2 = tmax;
    if (t1 >= t2) return false;
    if (t1 < 0.0f) t1 = 0.0f;
    float ray_length = length(r.d);
    float distance_inside = (t2 - t1) * ray_length;
    PROF_T0(pl);
    float hit_distance = cst(E)->neg_inv_density * rt_logf(std01(g, k));
    PROF_ADD(kPrLog, pl);
    if constexpr (kKind == 0 && kMediumFirst<kF>) {
        if (vbound < kInf) {  // t2 and the inside distance only grow with closest_so_far (monotone roundings)
            const float t2v = t2 > vbound ? vbound : t2;
            if (!(t1 < t2v) || hit_distance > (t2v - t1) * ray_length) replay = true;
        }
    }
    if (hit_distance > distance_inside) return false;
    t_out = t1 + hit_distance / ray_length;
    return true;
}

// ---------------------------------------------------------------------------
// HitRecord reconstruction (hittable.rs:28-52 + each primitive's tail)
// ---------------------------------------------------------------------------
struct Rec {
    V p, n;
    float t, u, v;
    bool front;
    uint32_t mat;
};
__device__ __noinline__ void sphere_uv(V p, float& u, float& v) {  // sphere.rs:41-46
    const float PI = 3.14159265358979323846f;
    const float TWO_PI = 2.0f * PI;
    float theta = rt_acosf(-p.y);
    float phi = rt_atan2f(-p.z, p.x) + PI;
    u = phi / TWO_PI;
    v = theta / PI;
}
RT_DEV void rec_new(Rec& rec, const Ray& r, V outward, float t, float u, float v, uint32_t mat) {
    rec.p = at(r, t);
    rec.front = sign_negative(dot(r.d, outward));
    rec.n = rec.front ? outward : -outward;
    rec.t = t;
    rec.u = u;
    rec.v = v;
    rec.mat = mat;
}
// (u, v) are computed only when the material reads them (kMatNeedsUV): they have
// no side effects, so skipping them elsewhere changes no bit of the output.
RT_DEV bool needs_uv(const DevScene& S, uint32_t mat) { return (S.mats[mat].flags & rtdev::kMatNeedsUV) != 0u; }
template <uint32_t kF = kFAll>
RT_DEV void prim_record(const DevScene& S, uint32_t code, const Ray& r, float t, Rec& rec) {
    uint32_t type = rtdev::leaf_type(code), idx = rtdev::leaf_index(code);
    float u = 0.0f, v = 0.0f;
    if (type == rtdev::kLeafSphere) {
        f4 s = ld4(S.sph + idx);
        uint32_t mat = S.sph_mat[idx];
        V p = at(r, t);
        V n = divs(p - xyz(s), s.w);
        if (needs_uv(S, mat)) sphere_uv(n, u, v);
        rec_new(rec, r, n, t, u, v, mat);
    } else if (type == rtdev::kLeafRect) {
        f4 r0 = ld4(S.rect + 2 * idx), r1 = ld4(S.rect + 2 * idx + 1);
        uint32_t axis = __float_as_uint(r1.y), mat = __float_as_uint(r1.z);
        if (needs_uv(S, mat)) {
            float ok, dk, oa, da, ob, db;
            rect_axes(axis, r, ok, dk, oa, da, ob, db);
            float x = oa + t * da, y = ob + t * db;
            u = (x - r0.y) / (r0.z - r0.y);
            v = (y - r0.w) / (r1.x - r0.w);
        }
        V n = axis == 0u ? mk(0.0f, 0.0f, 1.0f) : (axis == 1u ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f));
        rec_new(rec, r, n, t, u, v, mat);
    } else if ((kF & kFTri) && type == rtdev::kLeafTri) {
        f4 t0 = ld4(S.tri + 3 * idx), t1 = ld4(S.tri + 3 * idx + 1), t2 = ld4(S.tri + 3 * idx + 2);
        V n = normalize(cross(xyz(t1), xyz(t2)));
        rec_new(rec, r, n, t, 0.0f, 0.0f, __float_as_uint(t0.w));
    } else {  // moving sphere
        f4 m0 = ld4(S.msph + 3 * idx), m1 = ld4(S.msph + 3 * idx + 1), m2 = ld4(S.msph + 3 * idx + 2);
        uint32_t mat = __float_as_uint(m2.y);
        V p = at(r, t);
        V n = divs(p - msphere_center(m0, m1, m2, r.time), m0.w);
        if (needs_uv(S, mat)) sphere_uv(n, u, v);
        rec_new(rec, r, n, t, u, v, mat);
    }
}
template <uint32_t kF = kFAll>
RT_DEV void make_record(const DevScene& S, uint32_t entry, uint32_t code, float t, const Ray& r0, Rec& rec) {
    const DevEntry* E = S.entries + entry;
    uint32_t ntf = E->ntf;
    f4 op0 = E->tf[0], op1 = E->tf[1], op2 = E->tf[2];
    Ray r1 = ntf > 0u ? apply_op(op0, r0) : r0;
    Ray r2 = ntf > 1u ? apply_op(op1, r1) : r1;
    Ray r3 = ntf > 2u ? apply_op(op2, r2) : r2;
    if (rtdev::leaf_type(code) == rtdev::kLeafMedium) {  // hittable.rs:216-230
        rec.t = t;
        rec.p = at(r3, t);
        rec.n = mk(1.0f, 0.0f, 0.0f);
        rec.u = 0.0f;
        rec.v = 0.0f;
        rec.front = true;
        rec.mat = E->phase_mat;
    } else {
        prim_record<kF>(S, code, r3, t, rec);
    }
    // unwind the chain inner -> outer (instance.rs:41, 128-140)
#pragma unroll
    for (int i = 2; i >= 0; --i) {
        if ((uint32_t)i >= ntf) continue;
        f4 op = i == 0 ? op0 : (i == 1 ? op1 : op2);
        V dlev = i == 0 ? r1.d : (i == 1 ? r2.d : r3.d);  // the ray RotateY passed down
        if (op.w == 0.0f) {
            rec.p = rec.p + xyz(op);
        } else {
            float s = op.x, c = op.y;
            V p = mk(c * rec.p.x + s * rec.p.z, rec.p.y, -s * rec.p.x + c * rec.p.z);
            V n = mk(c * rec.n.x + s * rec.n.z, rec.n.y, -s * rec.n.x + c * rec.n.z);
            rec.p = p;
            bool ff = dot(dlev, n) < 0.0f;  // set_face_normal(&ray_rotated, normal)
            rec.n = ff ? n : -n;
        }
    }
}

// ---------------------------------------------------------------------------
// textures (src/textures/*) — Marble restates noise 0.8.2 Perlin/Turbulence
// ---------------------------------------------------------------------------
RT_DEV uint32_t perm_hash(const uint8_t* t, int64_t x, int64_t y, int64_t z) {
    uint32_t a = t[(uint32_t)(x & 0xff)];
    a = t[a ^ (uint32_t)(y & 0xff)];
    return t[a ^ (uint32_t)(z & 0xff)];
}
RT_DEV double surflet(uint32_t h, double dx, double dy, double dz) {
    const double D = 0.7071067811865476;
    double t = 1.0 - ((dx * dx + dy * dy) + dz * dz) * 2.0;
    if (!(t > 0.0)) return 0.0;
    uint32_t g = h % 12u;
    // grad3: (+-D, +-D, 0) for 0..3, (+-D, 0, +-D) for 4..7, (0, +-D, +-D) for 8..11
    double gx = g < 8u ? ((g & 2u) ? -D : D) : 0.0;
    double gy = g < 4u ? ((g & 1u) ? -D : D) : (g < 8u ? 0.0 : ((g & 2u) ? -D : D));
    double gz = g < 4u ? 0.0 : ((g & 1u) ? -D : D);
    double t2 = t * t;
    double t4 = t2 * t2;
    return (2.0 * t2 + t4) * ((dx * gx + dy * gy) + dz * gz);
}
RT_DEV double perlin3(const uint8_t* t, double px, double py, double pz) {
    const double SCALE = 1.1547005383792515;
    double fx = __builtin_floor(px), fy = __builtin_floor(py), fz = __builtin_floor(pz);
    int64_t ix = (int64_t)fx, iy = (int64_t)fy, iz = (int64_t)fz;
    double dx = px - fx, dy = py - fy, dz = pz - fz;
    double ex = dx - 1.0, ey = dy - 1.0, ez = dz - 1.0;
    double r = surflet(perm_hash(t, ix, iy, iz), dx, dy, dz);
    r = r + surflet(perm_hash(t, ix + 1, iy, iz), ex, dy, dz);
    r = r + surflet(perm_hash(t, ix, iy + 1, iz), dx, ey, dz);
    r = r + surflet(perm_hash(t, ix + 1, iy + 1, iz), ex, ey, dz);
    r = r + surflet(perm_hash(t, ix, iy, iz + 1), dx, dy, ez);
    r = r + surflet(perm_hash(t, ix + 1, iy, iz + 1), ex, dy, ez);
    r = r + surflet(perm_hash(t, ix, iy + 1, iz + 1), dx, ey, ez);
    r = r + surflet(perm_hash(t, ix + 1, iy + 1, iz + 1), ex, ey, ez);
    r = r * SCALE;
    if (r < -1.0) r = -1.0;
    if (r > 1.0) r = 1.0;
    return r;
}
RT_DEV double fbm_get(const uint8_t* tabs, uint32_t seed0, double x, double y, double z) {
    const double lacunarity = 3.141592653589793 * 2.0 / 3.0;
    double denom = 0.0, pw = 1.0;
    for (int i = 1; i <= 6; ++i) {
        pw = pw * 0.5;
        denom = denom + pw;
    }
    const double scale_factor = 1.0 / denom;
    double result = 0.0, persist = 1.0;
    x = x * 1.0; y = y * 1.0; z = z * 1.0;
    for (uint32_t o = 0; o < 6u; ++o) {
        double signal = perlin3(tabs + 256u * (1u + seed0 + o), x, y, z);
        signal = signal * persist;
        result = result + signal;
        persist = persist * 0.5;
        x = x * lacunarity; y = y * lacunarity; z = z * lacunarity;
    }
    return result * scale_factor;
}
__device__ __noinline__ double turbulence(const uint8_t* tabs, double px, double py, double pz) {
    const double power = 1.0;
    double xd = px + fbm_get(tabs, 0u, px + 12414.0 / 65536.0, py + 65124.0 / 65536.0, pz + 31337.0 / 65536.0) * power;
    double yd = py + fbm_get(tabs, 1u, px + 26519.0 / 65536.0, py + 18128.0 / 65536.0, pz + 60493.0 / 65536.0) * power;
    double zd = pz + fbm_get(tabs, 2u, px + 53820.0 / 65536.0, py + 11213.0 / 65536.0, pz + 44845.0 / 65536.0) * power;
    return perlin3(tabs, xd, yd, zd);
}
// The turbulence noise 0.8.2 computes for Marble (marble.rs:23-29) at p for every lane
// with `need`, evaluated by the whole wave together; all 64 lanes must call it
// (convergent). Sequentially it is 19 Perlin evaluations per lane, and a Marble hit
// is rare (3.4 lanes of 64 on C3): here the 18 fbm octaves (3 fbm x 6, independent
// of each other) of up to 3 requesting lanes are spread over 54 lanes, each lane
// evaluating one perlin3 with the same operations fbm_get applies for that octave
// (the point scaled by the lacunarity o times, then signal * persist, a power of
// two), the requester sums its octaves in fbm_get's order, and only the final
// perlin3 runs per lane. Every value is the one turbulence() computes, bit for bit.
// `tab` = the Marble's first permutation table (DevTexture::a).
__device__ __forceinline__ double turbulence_wave(const uint8_t* perm, bool need, V p, uint32_t tab) {
    const uint32_t lane = __lane_id();
    unsigned long long pending = __ballot(need);
    double xd = 0.0, yd = 0.0, zd = 0.0;
    const double lac = 3.141592653589793 * 2.0 / 3.0;
    double denom = 0.0, pw = 1.0;
    for (int i = 1; i <= 6; ++i) {
        pw = pw * 0.5;
        denom = denom + pw;
    }
    const double scale_factor = 1.0 / denom;
    const uint32_t j = lane / 18u, k = lane - j * 18u, f = k / 6u, o = k - f * 6u;  // this lane's (requester, fbm, octave)
    while (pending) {
        uint32_t req[3] = {0u, 0u, 0u}, nreq = 0u;
        for (; nreq < 3u && pending; ++nreq) {
            req[nreq] = (uint32_t)__builtin_ctzll(pending);
            pending &= pending - 1ull;
        }
        const uint32_t src = j == 0u ? req[0] : (j == 1u ? req[1] : req[2]);
        const float qx = __shfl(p.x, (int)src), qy = __shfl(p.y, (int)src), qz = __shfl(p.z, (int)src);
        const uint32_t qt = __shfl(tab, (int)src);
        double sig = 0.0;
        if (j < nreq) {  // fbm_get(tabs, f, p + offset_f) octave o
            const double ox = f == 0u ? 12414.0 / 65536.0 : (f == 1u ? 26519.0 / 65536.0 : 53820.0 / 65536.0);
            const double oy = f == 0u ? 65124.0 / 65536.0 : (f == 1u ? 18128.0 / 65536.0 : 11213.0 / 65536.0);
            const double oz = f == 0u ? 31337.0 / 65536.0 : (f == 1u ? 60493.0 / 65536.0 : 44845.0 / 65536.0);
            double x = (double)qx + ox, y = (double)qy + oy, z = (double)qz + oz;
            x = x * 1.0; y = y * 1.0; z = z * 1.0;
            double persist = 1.0;
            for (uint32_t i = 0; i < o; ++i) {
                persist = persist * 0.5;
                x = x * lac; y = y * lac; z = z * lac;
            }
            sig = perlin3(perm + 256u * (qt + 1u + f + o), x, y, z) * persist;
        }
        // requester r of this round sums its 18 signals in fbm_get's order
        int mine = -1;
        for (uint32_t r = 0; r < nreq; ++r)
            if (lane == req[r]) mine = (int)r;
        double fb[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (uint32_t ff = 0; ff < 3u; ++ff) {
            double result = 0.0;
#pragma unroll
            for (uint32_t oo = 0; oo < 6u; ++oo) {
                const int from = (mine < 0 ? 0 : mine) * 18 + (int)(ff * 6u + oo);
                const double v = __shfl(sig, from);
                result = result + v;
            }
            fb[ff] = result * scale_factor;
        }
        if (mine >= 0) {
            const double power = 1.0;
            xd = (double)p.x + fb[0] * power;
            yd = (double)p.y + fb[1] * power;
            zd = (double)p.z + fb[2] * power;
        }
    }
    return need ? perlin3(perm + 256u * tab, xd, yd, zd) : 0.0;
}

// The texture a chain of Checkers (checker.rs:27-37) resolves to at p: what tex_value
// would evaluate. Side-effect free, so tex_value may start from the result (same bits).
RT_DEV uint32_t tex_resolve(const DevScene& S, uint32_t tid, V p) {
    for (;;) {
        const DevTexture* T = S.texs + tid;
        if (T->kind != rtdev::kTexChecker) return tid;
        float sc = T->scale;
        float sines = rt_sinf(sc * p.x) * rt_sinf(sc * p.y) * rt_sinf(sc * p.z);
        tid = sign_negative(sines) ? T->b : T->a;
    }
}

// kTurb: a Marble reached by this evaluation takes `turb` (turbulence_wave's value at the
// same p) instead of computing the turbulence itself.
template <bool kTurb = false>
RT_DEV V tex_value(const DevScene& S, uint32_t tid, float u, float v, V p, double turb = 0.0) {
    for (;;) {
        const DevTexture* T = S.texs + tid;
        uint32_t kind = T->kind;
        if (kind == rtdev::kTexSolid) return mk(T->color[0], T->color[1], T->color[2]);  // solid_color.rs:21-25
        if (kind == rtdev::kTexChecker) {                                                  // checker.rs:27-37
            PROF_T0(pc);
            float sc = T->scale;
            float sines = rt_sinf(sc * p.x) * rt_sinf(sc * p.y) * rt_sinf(sc * p.z);
            tid = sign_negative(sines) ? T->b : T->a;
            PROF_ADD(kPrChecker, pc);
            continue;
        }
        if (kind == rtdev::kTexMarble) {  // marble.rs:23-29
            PROF_T0(pm);
            double n = kTurb ? turb : turbulence(S.perm + 256u * T->a, (double)p.x, (double)p.y, (double)p.z);
            float s = 0.5f * (1.0f + rt_sinf(T->scale * p.z + 10.0f * (float)n));
            PROF_ADD(kPrMarble, pm);
            return mk(s, s, s);
        }
        PROF_T0(pi);
        // image_texture.rs:21-52
        uint32_t w = T->b, h = T->c;
        float uu = rs_clamp(u, 0.0f, 1.0f);
        float vv = 1.0f - rs_clamp(v, 0.0f, 1.0f);
        uint32_t i = rt_f32_to_u32_sat(uu * (float)w);
        uint32_t j = rt_f32_to_u32_sat(vv * (float)h);
        if (i >= w) i = w - 1u;
        if (j >= h) j = h - 1u;
        const uint8_t* px = S.texels + T->a + ((size_t)j * w + i) * 3u;
        const float cs = 1.0f / 255.0f;
        V texel = mk((float)px[0] * cs, (float)px[1] * cs, (float)px[2] * cs);
        PROF_ADD(kPrImage, pi);
        return texel;
    }
}

// ---------------------------------------------------------------------------
// materials (src/materials/*)
// ---------------------------------------------------------------------------
RT_DEV V reflect(V v, V n) { return v - (2.0f * dot(v, n)) * n; }  // utils.rs:37-39
RT_DEV V refract(V uv, V n, float eta) {                          // utils.rs:41-46
    float cos_t = rs_min(dot(-uv, n), 1.0f);
    V r_perp = eta * (uv + cos_t * n);
    V r_par = (-__builtin_sqrtf(__builtin_fabsf(1.0f - dot(r_perp, r_perp)))) * n;
    return r_par + r_perp;
}
RT_DEV bool near_zero(V v) {  // utils.rs:5-7
    const float eps = 1.1920929e-07f;
    return __builtin_fabsf(v.x) < eps && __builtin_fabsf(v.y) < eps && __builtin_fabsf(v.z) < eps;
}
// att_later: the caller evaluates a Marble attenuation itself (after the wave-wide turbulence).
template <bool kTurb = false>
RT_DEV bool scatter(const DevScene& S, const DevMaterial& m, const Ray& r, const Rec& rec, Rng& g, const Key& k,
                    V& att, Ray& sc, uint32_t tex = 0u, double turb = 0.0, bool att_later = false) {
    sc.o = rec.p;
    sc.time = r.time;
    // Lambertian, Metal and Isotropic each draw exactly one in_unit_sphere() and
    // nothing else (lambertian.rs:36, metal.rs:30, isotropic.rs:37): draw it once here.
    V rs = mk(0.0f, 0.0f, 0.0f);
    if (m.kind == rtdev::kMatLambertian || m.kind == rtdev::kMatMetal || m.kind == rtdev::kMatIsotropic) {
        PROF_T0(pu);
        rs = in_unit_sphere(g, k);
        PROF_ADD(kPrUnitSphere, pu);
#ifdef RT_DEBUG_PIXEL
        if ((RT_DEBUG_TRACE & 2) && g.pixel == RT_DEBUG_PIXEL && g.sample == RT_DEBUG_SAMPLE)
            dbg_put(2u, __float_as_uint(rs.x), __float_as_uint(rs.y), __float_as_uint(rs.z), g.d, g.r0, g.r1, g.r2);
#endif
    }
    if (m.kind == rtdev::kMatLambertian) {  // lambertian.rs:34-53
        PROF_T0(pb);
        V dir = rec.n + normalize(rs);
        if (near_zero(dir)) dir = rec.n;
        sc.d = dir;
        if (!att_later) att = tex_value<kTurb>(S, kTurb ? tex : m.tex, rec.u, rec.v, rec.p, turb);
        PROF_ADD(kPrLambert, pb);
        return true;
    }
    if (m.kind == rtdev::kMatMetal) {  // metal.rs:25-43
        PROF_T0(pt);
        V reflected = reflect(normalize(r.d), rec.n);
        V dir = reflected + m.fuzz * rs;
        sc.d = dir;
        att = mk(m.albedo[0], m.albedo[1], m.albedo[2]);
        PROF_ADD(kPrMetal, pt);
        return dot(dir, rec.n) > 0.0f;
    }
    if (m.kind == rtdev::kMatDielectric) {  // dialectric.rs:32-61
        PROF_T0(pd);
        att = mk(1.0f, 1.0f, 1.0f);
        float ratio = rec.front ? 1.0f / m.ior : m.ior;
        V ud = normalize(r.d);
        float cos_t = rs_min(dot(-ud, rec.n), 1.0f);
        float sin_t = __builtin_sqrtf(1.0f - cos_t * cos_t);
        bool cannot = ratio * sin_t > 1.0f;
        bool refl = cannot;
        if (!cannot) {
            float q = (1.0f - ratio) / (1.0f + ratio);  // Schlick, dialectric.rs:26-29
            float r0 = q * q;
            float x = 1.0f - cos_t;
            float x2 = x * x;
            float refl_p = r0 + (1.0f - r0) * (x * (x2 * x2));
            refl = refl_p > std01(g, k);
        }
        sc.d = refl ? reflect(ud, rec.n) : refract(ud, rec.n, ratio);
        PROF_ADD(kPrDielectric, pd);
        return true;
    }
    if (m.kind == rtdev::kMatIsotropic) {  // isotropic.rs:31-43
        PROF_T0(ps);
        sc.d = rs;
        if (!att_later) att = tex_value<kTurb>(S, kTurb ? tex : m.tex, rec.u, rec.v, rec.p, turb);
        PROF_ADD(kPrIso, ps);
        return true;
    }
    return false;  // DiffuseLight never scatters (diffuse_light.rs:26-32)
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
RT_DEV void start_sample(const DevCamera& C, const DevParams& P, const Key& k, uint32_t x, uint32_t y,
                         uint32_t pixel, uint32_t sample, Rng& g, Ray& ray) {
    g.sample = sample;
    g.pixel = pixel;
    g.d = 0u;
    // renderer.rs:141-142
    float u = ((float)x + std01(g, k)) / (float)(P.width - 1u);
    float v = ((float)y + std01(g, k)) / (float)(P.height - 1u);
    // camera.rs:96-106
    V rd = C.lens_radius * in_unit_disk(g, k);
    V cu = mk(C.u[0], C.u[1], C.u[2]), cv = mk(C.v[0], C.v[1], C.v[2]);
    V org = mk(C.origin[0], C.origin[1], C.origin[2]);
    V offset = rd.x * cu + rd.y * cv;
    ray.o = org + offset;
    V llc = mk(C.llc[0], C.llc[1], C.llc[2]);
    V hor = mk(C.horizontal[0], C.horizontal[1], C.horizontal[2]);
    V ver = mk(C.vertical[0], C.vertical[1], C.vertical[2]);
    ray.d = llc + u * hor + v * ver - org - offset;
    float v01 = from_1_2(next_u32(g, k)) - 1.0f;  // gen_range(t0..=t1)
    ray.time = v01 * C.time_scale + C.time_low;
}

// One launch covers samples [sample0, sample0 + samples) of every pixel of the shard.
// Work units are (8x8 block, sample) pairs, block-major; a batch is up to `group` consecutive
// units (64 items each) that a wave takes with one atomic and feeds to its idle lanes.
// The best batch size follows the work per wave: the power of two at or below 1/64 of the
// units each resident wave will process, within [4, 16]. Measured on C3 (same box, units per
// wave -> ms per launch for batch sizes): 1831 (500 spp, one GPU) -> 16: 511, 8: 518, 32: 540;
// 915 (250 spp, or one rank of two) -> 8: 264, 12: 270, 16: 278; 458 (rank of four) -> 4: 138,
// 8: 144; 366 (100 spp) -> 4: 112, 8: 119; 230 (63 spp, or one rank of eight) -> 2: 77, 4: 74,
// 8: 82, 16: 97. The fixed 16 cost an 8-GPU rank a third of its time.
// Round 5 (same box, 500-spp C3 shards, tools/shard_time.py, RT_GROUP sweep): the batches in flight
// (waves x group units, block-major) span group / (units per wave) of the shard's blocks, and a
// shard's blocks span the whole image; a rank slows down steeply once that window passes ~4% of
// the image (one rank of 8, 261 units per wave: group 4 57.1 ms, 8 55.5, 10 55.4, 12 60.1, 16 68.6;
// of 16: 4 30.9, 6 32.3, 8 36.3) and gains a little from larger batches below it (rank of 4:
// 8 107.9, 16 106.5; one GPU: 16 415.3, 24 413.1). The flat and triangle presets gain more
// (one GPU: C5 946 -> 905 ms with 64, C4 1461 -> 1449). So: a 1/32 window, 4..64 units.
static inline uint32_t batch_group(uint64_t units, uint32_t waves) {
    const uint64_t g = units / ((uint64_t)(waves ? waves : 1u) * 32u);
    return g < 4u ? 4u : g > 64u ? 64u : (uint32_t)g;
}
constexpr uint32_t kPermLdsMax = 4u * 9u * 256u;  // up to four Marble textures staged in LDS
#ifndef RT_MT_LDS
#define RT_MT_LDS 1
#endif
constexpr uint32_t kMtLdsMax = 2048u;  // material + texture records staged in LDS by the flat-list preset
struct ChunkParams {
    uint32_t sample0;         // global sample index of chunk sample 0 (includes P.sample_base)
    uint32_t samples;         // samples per pixel in this chunk
    uint32_t units;           // work units: (8x8 block of the shard, sample) pairs, block-major
    uint32_t guide;           // the guided batch divisor: a batch is at most rem / (guide x waves) units
    uint32_t fast_grid;       // waves of the fast kernel's launch (the streaming replay pass waits for them)
    uint32_t nslots;          // sample-buffer plane size: 64 slots per 8x8 block of the shard, block-major
    uint32_t group;           // units per batch at most (batch_group)
    uint32_t blocks;          // 8x8 blocks of the shard (units = blocks x samples)
};

// HittableList::hit over the world (hittable.rs:100-118), t in [0.001, inf).
template <int kKind, uint32_t kF>
RT_DEV bool world_hit(const DevScene& S, float delta, const Ray& r, Rng& g, const Key& k, float& t_hit,
                      uint32_t& hit_entry, uint32_t& hit_code, uint32_t* stk, uint32_t mode, bool& replay) {
    float closest = kInf;
    float cb = kInf;  // the medium-first bound C (medium_first_estimate)
    if constexpr (kKind == 0 && kMediumFirst<kF>) {
        // (every wave takes the bound: bounding only the waves with few active lanes, the drain's,
        // gained nothing over no bound)
        if (S.mb_entry < S.num_top) {
            cb = medium_first_estimate<kF>(S, S.entries + S.mb_entry, r, g, k);
#ifdef RT_LEAF_AUDIT
            // audit build, RT_OPT_TUNE kModeMbShrink: an estimate half as far, so that the exact check
            // fails wherever the walk finds nothing below it and the fallback (the hand-over) is exercised
            if (mode & kModeMbShrink) cb *= 0.5f;
#endif
            // B = C(1 + 2^-18) + 2 delta / min|d_a|: bvh_hit's inflated-entry margin te - delta * max|inv_a|
            // (the BVHs before the medium are translated only, so the ray's inverse direction is
            // theirs; the factor 2 and the 2^-18 cover the roundings of inv and of B itself)
            const float md = fminf(fabsf(r.d.x), fminf(fabsf(r.d.y), fabsf(r.d.z)));
            const float b = cb * (1.0f + 0x1p-18f) + (delta + delta) / md;
            if (b < kInf) closest = b; else cb = kInf;
        }
    }
    bool any = false;
    for (uint32_t e = 0; e < S.num_top; ++e) {
        const DevEntry* E = S.entries + e;
        PROF_T0(pe);
        if (uni<kF>(cst(E)->kind) == rtdev::kEntMedium) {
            float t, vb = kInf;
            if constexpr (kKind == 0 && kMediumFirst<kF>) {
                if (e == S.mb_entry && closest > cb) {  // nothing <= C before the medium: enter it with inf
                    closest = kInf;
                    any = false;
                    vb = cb;
                }
            }
            const bool mh = medium_hit<kKind, kF>(S, delta, E, r, 0.001f, closest, g, k, t, stk, mode, replay, vb);
            if (vb < kInf && !mh) replay = true;  // the estimate's scatter point did not hold
            if (mh) {
                closest = t;
                hit_entry = e;
                hit_code = rtdev::leaf_code(rtdev::kLeafMedium, 0);
                any = true;
            }
        } else {
            uint32_t code;
            if (entry_geom_hit<kKind, kF>(S, delta, E, r, 0.001f, closest, code, stk, mode, replay)) {
                hit_entry = e;
                hit_code = code;
                any = true;
            }
        }
        PROF_ADD(e < kPrEntryLast - kPrEntry0 ? kPrEntry0 + e : kPrEntryLast, pe);
    }
    t_hit = closest;
    return any;
}

// The suspending list walk of the fast kernel (instances with kFSusp): hittable.rs:100-118 per lane from
// its own position. A lane's walk state survives the trips of the sample loop: when a BVH
// traversal is suspended (bvh_run<.., true>: at most `susp` lanes of the wave were left in
// it), the lane stops its walk there, the others finish theirs and shade, and on the next
// trip the suspended lanes resume that traversal together with the lanes whose new
// segment reaches the same BVH. The long traversal tails, which ran at a few active lanes,
// then share their visits with fresh traversals. Each lane still visits the entries in list
// order with the same closest_so_far, and draws the medium's ln(U) where the reference does.
struct Walk {
    uint32_t pos;        // next entry of the segment's walk; num_top once the walk is complete
    bool resume;         // entry `pos` is a BVH whose traversal is suspended in tv
    bool any;            // hittable.rs:104 hit_anything
    float closest;       // hittable.rs:106 closest_so_far
    uint32_t hit_entry, hit_code;
    Trav tv;
};
template <uint32_t kF>
RT_DEV void world_walk(const DevScene& S, float delta, const Ray& ray, Rng& g, const Key& k, Walk& w, bool active,
                       uint32_t* stk, uint32_t mode, bool& replay, uint32_t susp) {
    for (uint32_t e = 0; e < S.num_top; ++e) {
        if (!(active && w.pos == e)) continue;
        PROF_T0(pe);
        const DevEntry* E = S.entries + e;
        const uint32_t kind = uni<kF>(cst(E)->kind);
        if (kind == rtdev::kEntMedium) {
            float t;
            if (medium_hit<0, kF>(S, delta, E, ray, 0.001f, w.closest, g, k, t, stk, mode, replay)) {
                w.closest = t;
                w.hit_entry = e;
                w.hit_code = rtdev::leaf_code(rtdev::kLeafMedium, 0);
                w.any = true;
            }
            w.pos = e + 1u;
        } else if ((kF & kFBvh) && kind == rtdev::kEntBvh) {
            Ray r = ray;
            const uint32_t ntf = uni<kF>(cst(E)->ntf);
            for (uint32_t i = 0; i < ntf; ++i) r = apply_op_u<kF>(ld4c(&E->tf[i]), r);
            const uint32_t root = uni<kF>(cst(E)->payload);
            const f4* wrapper = S.nodes + (size_t)root * rtdev::kBvhNodeF4;
            const V inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
            if (!w.resume) {  // bvh_hit's hand-over rule (NaN-prone rays go to the reference kernel)
                const uint32_t route = ray_route<0, kF>(r, inv, w.closest, wrapper, mode);
                if constexpr (RT_TRI_ZERO_DIR_FAST && (kF & kFTri) != 0u) {
                    if (route == kRayNoHit) {  // a NaN ray: the mesh returns no hit (bvh_hit's answer)
                        w.pos = e + 1u;
                        continue;
                    }
                }
                if (route != kRayFast) {
                    replay = true;
                    w.pos = S.num_top + 1u;  // abandoned: the sample is re-traced by the reference kernel
                    continue;
                }
                w.tv = Trav{root, 0u, 0u, w.closest, false, kNoNode};
            }
            if (bvh_run<0, kF, true>(S, delta, wrapper, r, inv, 0.001f, w.closest, w.hit_code, stk, mode, w.tv, susp)) {
                trav_audit(S, wrapper, root, r, inv, 0.001f, w.tv, w.closest, w.hit_code, stk);
                if (w.tv.any) {
                    w.hit_entry = e;
                    w.any = true;
                }
                w.pos = e + 1u;
                w.resume = false;
            } else {
                w.resume = true;
            }
        } else {
            uint32_t code;
            if (entry_geom_hit<0, kF>(S, delta, E, ray, 0.001f, w.closest, code, stk, mode, replay)) {
                w.hit_entry = e;
                w.hit_code = code;
                w.any = true;
            }
            w.pos = e + 1u;
        }
        PROF_ADD(e < kPrEntryLast - kPrEntry0 ? kPrEntry0 + e : kPrEntryLast, pe);
    }
}

// Renderer::get_color's sample loop (renderer.rs:140-146) as a work pool. Each
// lane owns one camera sample at a time; when its path ends (ray.rs:32-62) it
// stores the sample's radiance in the HBM sample buffer and takes the next item.
// Idle lanes are refilled with a wave ballot + mbcnt from a wave-local batch, and
// a batch costs one atomic, so no lane waits for a neighbour's long path.
// resolve_samples() then sums every pixel's samples IN SAMPLE ORDER, exactly like
// `color_accumulator +=` in the reference.
struct ItemPool {  // wave-uniform
    uint32_t batch, next, end;  // batch = its first unit; next / end: items (64 per unit) of the batch
    bool exhausted;
};
// Per-chunk device counters of the trace stage (zeroed before each chunk).
struct TraceCounters {
    unsigned batch;              // next 8x8-block batch of the fast (or exact) kernel
    unsigned replay_count;       // samples handed to the reference kernel
    unsigned replay_pull;        // next replay-list entry (reference kernel)
    unsigned batch_full;         // next batch when the replay list overflowed
    unsigned fast_done;          // fast-kernel waves that have finished (the streaming replay's end)
    unsigned stream_abort;       // the streaming replay gave up a claimed entry: re-render the chunk
    unsigned long long fast_segments;  // segments of the fast kernel's and streaming replay's samples
};
// A replay-list entry: the sample's pixel and its chunk-local sample index. Entries are
// written and read as one 64-bit agent-scope atomic: the streaming replay pass reads them
// while the fast kernel still runs, on other XCDs. A free entry holds kReplayFree.
struct ReplayItem {
    uint32_t pixel, sample;
};
constexpr unsigned long long kReplayFree = ~0ull;
constexpr size_t kCamOffset = 256;  // RT_CAMMEM: byte offset of the launch's DevCamera copy behind the counters
RT_DEV void replay_publish(ReplayItem* list, uint32_t idx, uint32_t pixel, uint32_t sample) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(list + idx),
                       (unsigned long long)pixel | ((unsigned long long)sample << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
RT_DEV unsigned long long replay_peek(const ReplayItem* list, uint32_t idx) {
    return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(list + idx), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}
// Takes entry idx and frees it for the next chunk.
RT_DEV ReplayItem replay_take(const ReplayItem* list, uint32_t idx) {
    const unsigned long long v = replay_peek(list, idx);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(const_cast<ReplayItem*>(list) + idx), kReplayFree,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return ReplayItem{(uint32_t)v, (uint32_t)(v >> 32)};
}
constexpr uint32_t kReplayCap = 1u << 20;
// A finished sample's radiance into the sample buffer (read once, by resolve_samples). RT_SBUF_NT:
// non-temporal stores, so the 5.76 GB a C3 frame streams through do not evict the hot lines (scene
// rows, register spills) from L2. Measured (same box, 100-spp C3 / 50-spp C4 frames): C3 79.15 ->
// 78.85 ms and 12.3 -> 8.9 GB of HBM traffic, C4 61.7 -> 61.6 ms and 63.8 -> 58.3 GB
// (profiles/r06/experiments/sample_buffer_nt_and_waves_*). The flat-list presets (C2, C5) keep plain
// stores: there the non-temporal form doubled the sample buffer's HBM writes (C2 7.5 -> 11.8 GB,
// C5 83 -> 118 GB per frame: 12-byte records written around L2) at equal speed
// (mc_schedulers_and_nt_bvh_only_ab.log). RT_SBUF_NT 2: non-temporal in the BVH presets only (the
// product); 1: every preset; 0: plain stores everywhere (A/B).
#ifndef RT_SBUF_NT
#define RT_SBUF_NT 2
#endif
template <uint32_t kF = kFAll>
RT_DEV void sbuf_store(float* o, V L) {
    if constexpr (RT_SBUF_NT == 1 || (RT_SBUF_NT == 2 && (kF & kFBvh) != 0u)) {
        __builtin_nontemporal_store(L.x, o);
        __builtin_nontemporal_store(L.y, o + 1);
        __builtin_nontemporal_store(L.z, o + 2);
    } else {
        o[0] = L.x;
        o[1] = L.y;
        o[2] = L.z;
    }
}
// The streaming replay pass (trace_samples<3> with fixup 2, on a second stream) claims
// entries one at a time while the fast kernel drains. Returns the claimed entry's index once
// it is published, or kReplayNone when the fast kernel finished without one, the list
// overflowed, or the wait timed out (then the serialized pass re-renders the chunk).
constexpr uint32_t kReplayNone = 0xffffffffu;
constexpr uint32_t kStreamWaves = 512;  // waves of the streaming replay pass
constexpr unsigned long long kStreamTimeoutTicks = 1000000000ull;  // 10 s of s_memrealtime (100 MHz)
RT_DEV uint32_t replay_claim(TraceCounters* ctr, const ReplayItem* list, uint32_t fast_grid) {
    const uint32_t i = atomicAdd(&ctr->replay_pull, 1u);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        // fast_done first: once every fast wave has counted itself out (after a release
        // fence), replay_count is final
        const bool done = __hip_atomic_load(&ctr->fast_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= fast_grid;
        const uint32_t n = __hip_atomic_load(&ctr->replay_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (i < n) {
            if (i >= kReplayCap) return kReplayNone;
            if (replay_peek(list, i) != kReplayFree) return i;
        } else if (done) {
            return kReplayNone;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > kStreamTimeoutTicks) {
            atomicExch(&ctr->stream_abort, 1u);
            return kReplayNone;
        }
        for (int z = 0; z < 4; ++z)  // ~32k cycles between polls: the pollers must not crowd the drain
            __builtin_amdgcn_s_sleep(127);
    }
}
// Gives the next work item to every lane with `want` set. A lane that got a
// sample returns true with its camera ray started (renderer.rs:141-143); a
// max_depth 0 sample (ray.rs:39-41: black, no segment) is stored and skipped.
// With `list` set, the items are that many replay-list entries instead (pulled
// through *counter in shares of ceil(list_n / waves), at most 64: the replayed
// paths are few and long, and a wave's segment takes as long as its slowest lane).
RT_DEV bool take_sample(ItemPool& pool, bool want, const DevCamera& C, const DevParams& P, const ChunkParams& Q,
                        const Key& k, unsigned* counter, const ReplayItem* list, uint32_t list_n,
                        TraceCounters* ctr, uint32_t stream_grid, float* sbuf,
                        uint32_t lane, uint32_t& slot, uint32_t& s_local, V& L, V& T, uint32_t& depth, Rng& g,
                        Ray& ray) {
    bool got = false;
#ifdef RT_LEAF_AUDIT
    if (__ballot(1) != ~0ull) atomicAdd(&g_bounds_audit_count, 1u);  // the whole wave must be here (leader)
#endif
    for (;;) {
        unsigned long long need = __ballot(want && !got);
        if (need == 0ull || pool.exhausted) break;
        if (pool.next == pool.end) {
            // Lane 0 claims and readfirstlane broadcasts: the same lane, because take_sample runs
            // with the whole wave active (every caller calls it at the top of its sample loop, in
            // uniform control flow, and a wave is one 64-thread workgroup). The audit build checks
            // that invariant at every entry (g_bounds_audit_count, asserted zero by the GPU suite).
            // Electing the first active lane instead (lane == ctz(ballot(1))) was measured: same
            // bits, but the register allocation it led to cost C3 3% and C4 4%.
            const bool leader = lane == 0u;
            // Guided batches: up to Q.group units while work is plentiful, shrinking with the
            // work left (rem / (2 x waves), at least one unit) so that the waves finish together
            // instead of the last ones draining a full batch alone.
            uint32_t bt = 0, cnt = 64u;
            if (list && stream_grid) {
                // The streaming replay keeps 1 + backlog / waves lanes of a wave busy: the
                // replayed paths are few and long, and a wave's segment takes as long as its
                // slowest lane, so they spread over the waves unless there are many.
                uint32_t lim = 1u;
                if (leader) {
                    const uint32_t n = __hip_atomic_load(&ctr->replay_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t pl = __hip_atomic_load(&ctr->replay_pull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    lim += (n > pl ? n - pl : 0u) / gridDim.x;
                }
                lim = __builtin_amdgcn_readfirstlane(lim);
                if (64u - (uint32_t)__popcll(need) >= lim) break;
            }
            if (leader) {
                if (list && stream_grid) {  // the streaming replay: one entry per claim
                    cnt = 1u;
                    bt = replay_claim(ctr, list, stream_grid);
#ifdef RT_PROFILE_REGIONS
                    role_event(bt);
#endif
                } else if (list) {  // a share of the list per wave: a replayed path runs with few others
                    cnt = (list_n + gridDim.x - 1u) / gridDim.x;
                    cnt = cnt > 64u ? 64u : cnt;
                    bt = atomicAdd(counter, cnt);
                } else {
                    const uint32_t cur = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint32_t rem = cur < Q.units ? Q.units - cur : 0u;
                    cnt = rem / (Q.guide * gridDim.x);
                    cnt = cnt < 1u ? 1u : (cnt > Q.group ? Q.group : cnt);
                    bt = atomicAdd(counter, cnt);
                }
            }
            bt = __builtin_amdgcn_readfirstlane(bt);
            cnt = __builtin_amdgcn_readfirstlane(cnt);
            if (bt >= (list ? list_n : Q.units)) {
                pool.exhausted = true;
                break;
            }
            pool.batch = bt;
            pool.next = list ? bt : 0u;
            pool.end = list ? (bt + cnt < list_n ? bt + cnt : list_n) : 64u * cnt;
            continue;
        }
        uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        uint32_t avail = pool.end - pool.next;
        if (want && !got && rank < avail) {
            uint32_t x, y, s, sl;
            if (list) {
                const ReplayItem it = replay_take(list, pool.next + rank);
                y = it.pixel / P.width;
                x = it.pixel - y * P.width;
                s = it.sample;
                const uint32_t blk = (y >> 3) * P.blocks_x + (x >> 3);
                sl = ((blk - P.shard_index) / P.shard_count) * 64u + ((y & 7u) << 3) + (x & 7u);
            } else {
                // unit pool.batch + (item >> 6); a batch (<= Q.group <= Q.samples units) crosses at
                // most one block boundary, so the batch's block and sample are divided once
                const uint32_t item = pool.next + rank;
                const uint32_t blk0 = __builtin_amdgcn_readfirstlane(pool.batch / Q.samples);
                const uint32_t s0 = pool.batch - blk0 * Q.samples;
                s = s0 + (item >> 6);
                uint32_t blk_local = blk0;
                if (s >= Q.samples) {
                    s -= Q.samples;
                    blk_local += 1u;
                }
                if (pool.batch + (item >> 6) >= Q.units) s = Q.samples;  // past the last unit: no work
                if (!(P.tune & kModeBlocksForward)) blk_local = Q.blocks - 1u - blk_local;
#ifdef RT_EXP_STRIDE
                if (P.tune & (1u << 23)) {  // A/B only: blocks in 8 interleave classes, one after another
                    uint32_t i = blk_local, r = 0u;
                    for (; r < 7u; ++r) {
                        const uint32_t cr = (Q.blocks - r + 7u) / 8u;
                        if (i < cr) break;
                        i -= cr;
                    }
                    blk_local = r + 8u * i;
                }
#endif
                uint32_t pib = item & 63u;
                sl = blk_local * 64u + pib;
                uint32_t blk = P.shard_index + blk_local * P.shard_count;
                uint32_t by = blk / P.blocks_x, bx = blk - by * P.blocks_x;
                x = bx * 8u + (pib & 7u);
                y = by * 8u + (pib >> 3);
            }
            if (x < P.width && y < P.height && s < Q.samples) {
                const uint32_t pixel = y * P.width + x;
                slot = sl;
                s_local = s;
                L = mk(0.0f, 0.0f, 0.0f);
                T = mk(1.0f, 1.0f, 1.0f);
                depth = P.max_depth;
                start_sample(C, P, k, x, y, pixel, Q.sample0 + s, g, ray);
                if (depth == 0u) {
                    sbuf_store(sbuf + ((size_t)s_local * Q.nslots + sl) * 3u, mk(0.0f, 0.0f, 0.0f));
                } else {
                    got = true;
                }
            }
        }
        uint32_t n = (uint32_t)__popcll(need);
        pool.next += n < avail ? n : avail;
    }
    return got;
}

// The end of a segment whose list walk is complete (ray.rs:43-61): background,
// or HitRecord + emit + scatter. Returns true when the path ends; its radiance is
// then stored in the sample buffer. (Instances with kFMarble do this inline in
// trace_samples, around the wave-wide turbulence.)
template <uint32_t kF = kFAll>
RT_DEV bool finish_segment(const DevScene& S, const DevParams& P, const ChunkParams& Q, const Key& k,
                           float* __restrict__ sbuf, bool any, uint32_t he, uint32_t hc, float t, Ray& ray, V& L, V& T,
                           uint32_t& depth, Rng& g, uint32_t slot, uint32_t s_local) {
    PROF_T0(pg);
#ifdef RT_DEBUG_PIXEL
    // diagnostic builds only (tools/trace_sample.py): RT_DEBUG_TRACE bit 1 records the segment's
    // entry (Rng state and hit), bit 2 the in_unit_sphere draw, bit 4 the scatter's result
    if ((RT_DEBUG_TRACE & 1) && g.pixel == RT_DEBUG_PIXEL && g.sample == RT_DEBUG_SAMPLE)
        dbg_put(1u, depth, g.d, g.r0, g.r1, g.r2, any ? hc : 0xffffffffu, __float_as_uint(t));
#endif
    bool done;
    if (!any) {
        L = L + T * mk(P.bg[0], P.bg[1], P.bg[2]);
        done = true;
    } else {
        Rec rec;
        PROF_T0(pc);
        make_record<kF>(S, he, hc, t, ray, rec);
        PROF_ADD(kPrRecord, pc);
        const DevMaterial m = S.mats[rec.mat];
        PROF_T0(pm);
        V em = m.kind == rtdev::kMatLight ? tex_value(S, m.tex, rec.u, rec.v, rec.p) : mk(0.0f, 0.0f, 0.0f);
        L = L + T * em;
        PROF_ADD(kPrEmit, pm);
        V att;
        Ray sc;
        PROF_T0(ps);
        bool scattered = scatter(S, m, ray, rec, g, k, att, sc);
        PROF_ADD(kPrScatter, ps);
#ifdef RT_DEBUG_PIXEL
        if ((RT_DEBUG_TRACE & 4) && g.pixel == RT_DEBUG_PIXEL && g.sample == RT_DEBUG_SAMPLE)
            dbg_put(3u, rec.mat, m.kind, __float_as_uint(sc.d.x), __float_as_uint(sc.d.y), __float_as_uint(sc.d.z), g.d,
                    __float_as_uint(rec.n.y));
#endif
        if (scattered) {
            T = T * att;
            ray = sc;
            depth -= 1u;
            done = depth == 0u;
        } else {
            done = true;
        }
    }
    if (done) {
        sbuf_store<kF>(sbuf + ((size_t)s_local * Q.nslots + slot) * 3u, L);
    }
    PROF_ADD(kPrSegment, pg);
    return done;
}

// The end of a segment (ray.rs:43-61) for instances with kFMarble: HitRecord, emission and
// scatter per lane, where a lane whose texture resolves to a Marble leaves only its
// attenuation (or, for a light, its emission) for after turbulence_wave, so the HitRecord
// is dead while the wave evaluates the turbulence together. The draws and every value are
// finish_segment's (the Marble value is tex_value's 0.5 * (1 + sin(scale * p.z + 10 * turb))).
// All 64 lanes must call it (turbulence_wave is convergent); lanes without `shade` only
// join the turbulence. Returns true when the lane's path ended (its sample is stored).
template <uint32_t kF>
RT_DEV bool shade_marble(const DevScene& S, const DevParams& P, const ChunkParams& Q, const Key& k,
                         float* __restrict__ sbuf, bool shade, bool any, uint32_t he, uint32_t hc, float t, Ray& ray,
                         V& L, V& T, uint32_t& depth, Rng& g, uint32_t slot, uint32_t s_local) {
    bool marble = false, mlight = false, scattered = false, done = false;
    V mp = mk(0.0f, 0.0f, 0.0f);
    uint32_t tab = 0u;
    float mscale = 0.0f;
    if (shade && !any) {  // ray.rs:45-47
        L = L + T * mk(P.bg[0], P.bg[1], P.bg[2]);
        done = true;
    } else if (shade) {
        Rec rec;
        PROF_T0(pc);
        make_record<kF>(S, he, hc, t, ray, rec);
        PROF_ADD(kPrRecord, pc);
        const DevMaterial m = S.mats[rec.mat];
        uint32_t tex = m.tex;
        if (m.kind == rtdev::kMatLight || m.kind == rtdev::kMatLambertian || m.kind == rtdev::kMatIsotropic) {
            tex = tex_resolve(S, m.tex, rec.p);
            const DevTexture& tx = S.texs[tex];
            marble = tx.kind == rtdev::kTexMarble;
            tab = tx.a;
            mscale = tx.scale;
        }
        mp = rec.p;
        mlight = m.kind == rtdev::kMatLight;
        if (!(marble && mlight)) {  // ray.rs:50 emitted (a Marble light's after the turbulence)
            const V em = mlight ? tex_value<true>(S, tex, rec.u, rec.v, rec.p, 0.0) : mk(0.0f, 0.0f, 0.0f);
            L = L + T * em;
        }
        V att;
        Ray sc;
        scattered = scatter<true>(S, m, ray, rec, g, k, att, sc, tex, 0.0, marble);
        if (scattered) {
            if (!marble) T = T * att;
            ray = sc;
            depth -= 1u;
            done = depth == 0u;
        } else {
            done = true;
        }
    }
    PROF_T0(pmw);
    const double turb = turbulence_wave(S.perm, marble, mp, tab);
    PROF_ADD(kPrMarble, pmw);
    if (marble) {  // marble.rs:23-29
        const float sv = 0.5f * (1.0f + rt_sinf(mscale * mp.z + 10.0f * (float)turb));
        if (mlight) L = L + T * mk(sv, sv, sv);
        else if (scattered) T = T * mk(sv, sv, sv);
    }
    if (shade && done) {
        sbuf_store<kF>(sbuf + ((size_t)s_local * Q.nslots + slot) * 3u, L);
    }
    return shade && done;
}

// Every live lane traces one whole segment per loop trip: the list walk with its
// BVH traversals inline, then finish_segment.
//
// trace_samples<0> is the fast kernel (BVH4, nearest-first, exact pruning).
// A sample whose ray could take a NaN hit in a BVH is handed to the reference
// kernel instead: it is dropped here (its partial segments uncounted) and listed
// in `replay`. trace_samples<1> traverses every BVH with the literal replay
// of bvh.rs; it renders whole chunks under RT_FLAG_EXACT_BVH (fixup == 0) and
// otherwise re-traces the listed samples from their camera ray (fixup == 1).
// Samples are independent and keyed by (pixel, global sample index), so the
// re-traced sample is exactly the reference's. Should the list overflow, the
// fixup kernel re-renders the whole chunk and takes back the fast kernel's
// segment count.
#ifndef RT_SUSPEND
#define RT_SUSPEND 24  // C4 at 3 waves, 50 spp: 8 129 ms, 16 112.4, 20 109.1, 24 108.0, 28 108.7, 32 111.1
#endif
constexpr uint32_t kSuspLanes = RT_SUSPEND;  // suspend a BVH traversal's tail at this many lanes or fewer
// kWaves: the waves per SIMD the register allocator must allow. 3 (<= 168 VGPRs)
// is the default; the fast kernel also exists at 4 (<= 128 VGPRs, a few spills),
// launched when the scene's LDS stack fits four waves per SIMD (rt_render_launch).
template <int kKind, int kWaves = 3, uint32_t kF = kFAll>
__global__ __launch_bounds__(64, kWaves) void trace_samples(DevScene Sg, DevCamera C, DevParams P, ChunkParams Q,
                                                    float* __restrict__ sbuf, TraceCounters* __restrict__ ctr,
                                                    ReplayItem* __restrict__ replay_list, uint32_t fixup,
                                                    unsigned long long* __restrict__ seg_counter) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t lane = threadIdx.x;
    uint32_t* stk = lds_stack + lane;  // [level][{node, t_enter}][lane]
    // Perlin permutation tables (Marble) behind the stack when they fit: the
    // three dependent byte lookups per lattice corner then hit LDS, not L2.
    DevScene S = Sg;
    if (S.perm_bytes != 0u && S.perm_bytes <= kPermLdsMax && !(P.tune & kModeNoPermLds)) {
        uint32_t* tab = lds_stack + S.stack_depth * 128u;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(Sg.perm);
        for (uint32_t i = lane; i < S.perm_bytes / 4u; i += 64u) tab[i] = src[i];
        __syncthreads();
        S.perm = reinterpret_cast<const uint8_t*>(tab);
    }
    if constexpr (kKind == 0 && (kF & (kFBvh | kFTri | kFMarble)) == 0u) {
        // The flat-list preset (C5): a small scene's materials and textures behind the stack, so the
        // per-lane material / texture reads of every shading step hit LDS instead of the vector memory
        // path (the region profile put C5's emission and texture steps, mostly those loads' waits, at 19%)
        if (S.mt_lds) {
            uint32_t* tab = lds_stack + S.stack_depth * 128u;
            const uint32_t nm = S.num_mats * (sizeof(DevMaterial) / 4u), nt = S.num_texs * (sizeof(DevTexture) / 4u);
            const uint32_t* sm = reinterpret_cast<const uint32_t*>(Sg.mats);
            const uint32_t* st = reinterpret_cast<const uint32_t*>(Sg.texs);
            for (uint32_t i = lane; i < nm; i += 64u) tab[i] = sm[i];
            for (uint32_t i = lane; i < nt; i += 64u) tab[nm + i] = st[i];
            __syncthreads();
            S.mats = reinterpret_cast<const DevMaterial*>(tab);
            S.texs = reinterpret_cast<const DevTexture*>(tab + nm);
        }
    }
    if (kKind == 2) {  // HRPP counters behind the stack and the Perlin tables
        const uint32_t perm_words =
            S.perm_bytes != 0u && S.perm_bytes <= kPermLdsMax && !(P.tune & kModeNoPermLds) ? S.perm_bytes / 4u : 0u;
        S.hrpp_cnt = lds_stack + S.stack_depth * 128u + perm_words;
        if (lane < 4u * S.hrpp_npred) S.hrpp_cnt[lane] = 0u;
        __syncthreads();
    }
    const Key k{P.seed_lo, P.seed_hi};
    const uint32_t mode = P.tune;
#ifdef RT_CAMMEM
    // the camera read from the device copy behind the counters at each new sample (not kept in
    // SGPRs across the loop); the by-value argument is the same values. Only the flat-list
    // preset's translation unit (kernel_flat.hip) is built this way: measured on the same box,
    // C5 124.3 vs 126.5 ms per 200-spp frame, while the BVH presets lose 1-1.3% with it (C2,
    // C3, C4; profiles/r04/experiments/camera_in_memory_ab_*.log).
    const DevCamera& Cs = *reinterpret_cast<const DevCamera*>(reinterpret_cast<const char*>(ctr) + kCamOffset);
#else
    const DevCamera& Cs = C;
#endif
    // item source: the chunk's block batches, or (fixup) the replay list
    unsigned* counter = &ctr->batch;
    const ReplayItem* list = nullptr;
    uint32_t list_n = 0u, stream_grid = 0u;
    if ((kKind == 1 || kKind == 3) && fixup == 2u) {
        // The streaming replay pass, beside the fast kernel on a second stream: its waves take
        // the slots the fast kernel's waves leave as it drains. One dispatched while the fast
        // kernel still has work gives its slot back at once.
        if (__hip_atomic_load(&ctr->batch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < Q.units) return;
        list = replay_list;
        list_n = kReplayCap;
        counter = &ctr->replay_pull;
        stream_grid = Q.fast_grid;
    } else if ((kKind == 1 || kKind == 3) && fixup) {
        const uint32_t n = __hip_atomic_load(&ctr->replay_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool abort = __hip_atomic_load(&ctr->stream_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
        if (n <= kReplayCap && !abort) {  // the entries the streaming pass (if any) did not take
            if (n == 0u) return;
            list = replay_list;
            list_n = n;
            counter = &ctr->replay_pull;
        } else {  // overflow: re-render the chunk; its segments replace the earlier passes'
            counter = &ctr->batch_full;
            for (uint32_t i = blockIdx.x * 64u + lane; i < kReplayCap; i += gridDim.x * 64u)
                (void)replay_take(replay_list, i);  // free the list for the next chunk
            if (blockIdx.x == 0u && lane == 0u && seg_counter)
                atomicAdd(seg_counter, 0ull - __hip_atomic_load(&ctr->fast_segments, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT));
        }
    }
    bool has = false;
    // A lane's pixel and chunk-local sample are its Rng's counter fields (start_sample sets
    // them), so they are not kept a second time; per-lane segment counts fit 32 bits.
    uint32_t slot = 0, take_sample_idx = 0, depth = 0;  // slot: the sample-buffer slot of the lane's pixel
    // A finished sample's segments are its scatters (max_depth - depth) plus, unless its last
    // scatter took depth to 0, the segment that ended it (background or no scatter).
    uint32_t nseg = 0;
    V L = mk(0.0f, 0.0f, 0.0f), T = mk(1.0f, 1.0f, 1.0f);
    Rng g{};
    Ray ray{};
    ItemPool pool{0u, 0u, 0u, false};
    PROF_INIT();
#ifdef RT_PROFILE_REGIONS
    const unsigned long long wave_t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t tp_bucket = 0u, tp_acc = 0u;
#endif
    if constexpr (kKind == 0 && (kF & kFSusp) != 0u) {  // the suspending walk (world_walk)
        Walk w{};
        w.pos = 0u;
        for (;;) {
            PROF_T0(pr);
            if (take_sample(pool, !has, Cs, P, Q, k, counter, list, list_n, ctr, stream_grid, sbuf, lane, slot, take_sample_idx, L, T, depth, g,
                            ray)) {
                has = true;
                w.pos = 0u;
                w.resume = false;
            }
            PROF_ADD(kPrRefill, pr);
            if (__ballot(has) == 0ull) break;  // pool exhausted and every path finished
            if (has && w.pos == 0u && !w.resume) {  // a new segment: ray.rs:43 world.hit(r, 0.001, inf)
                w.closest = kInf;
                w.any = false;
            }
            bool replay = false;
            PROF_T0(pw);
            world_walk<kF>(S, P.prune_delta, ray, g, k, w, has, stk, mode, replay, pool.exhausted ? 0u : kSuspLanes);
            PROF_ADD(kPrWorld, pw);
            if (has && replay) {  // hand the sample to the reference kernel
                unsigned idx = atomicAdd(&ctr->replay_count, 1u);
                if (idx < kReplayCap) replay_publish(replay_list, idx, g.pixel, g.sample - Q.sample0);
                has = false;
            }
            const bool walked = has && w.pos == S.num_top;
            if constexpr ((kF & kFMarble) != 0u) {
                if (shade_marble<kF>(S, P, Q, k, sbuf, walked, w.any, w.hit_entry, w.hit_code, w.closest, ray, L, T,
                                     depth, g, slot, g.sample - Q.sample0)) {
                    has = false;
                    nseg += P.max_depth - depth + (depth != 0u ? 1u : 0u);
                }
            } else if (walked && finish_segment<kF>(S, P, Q, k, sbuf, w.any, w.hit_entry, w.hit_code, w.closest, ray, L,
                                                    T, depth, g, slot, g.sample - Q.sample0)) {
                has = false;
                nseg += P.max_depth - depth + (depth != 0u ? 1u : 0u);
            }
            if (walked) w.pos = 0u;
        }
    } else
    for (;;) {
        PROF_T0(pr);
        if (take_sample(pool, !has, Cs, P, Q, k, counter, list, list_n, ctr, stream_grid, sbuf, lane, slot, take_sample_idx, L, T, depth, g,
                        ray)) {
            has = true;
        }
        PROF_ADD(kPrRefill, pr);
        if (__ballot(has) == 0ull) break;  // pool exhausted and every path finished
#ifdef RT_PROFILE_REGIONS
        if (kKind == 0) {  // throughput histogram: this iteration's segments into the current bucket
            const uint32_t b = (uint32_t)((__builtin_amdgcn_s_memrealtime() - wave_t0) / kTpTicks);
            if (b != tp_bucket) {
                if (lane == 0u && tp_acc && tp_bucket < kTpBuckets) atomicAdd(&g_tp_hist[tp_bucket], tp_acc);
                tp_bucket = b;
                tp_acc = 0u;
            }
            tp_acc += (uint32_t)__popcll(__ballot(has));
        }
#endif
        if constexpr ((kF & kFMarble) != 0u) {
            bool shade = false, any = false;
            float t = 0.0f;
            uint32_t he = 0, hc = 0;
            if (has) {
                bool replay = false;
                PROF_T0(pw);
                any = world_hit<kKind, kF>(S, P.prune_delta, ray, g, k, t, he, hc, stk, mode, replay);
                PROF_ADD(kPrWorld, pw);
                if (kKind == 0 && replay) {  // hand the sample to the reference kernel
                    unsigned idx = atomicAdd(&ctr->replay_count, 1u);
                    if (idx < kReplayCap) replay_publish(replay_list, idx, g.pixel, g.sample - Q.sample0);
                    has = false;
                } else {
                    shade = true;
                }
            }
            if (shade_marble<kF>(S, P, Q, k, sbuf, shade, any, he, hc, t, ray, L, T, depth, g, slot, g.sample - Q.sample0)) {
                has = false;
                nseg += P.max_depth - depth + (depth != 0u ? 1u : 0u);
            }
        } else if (has) {
            float t;
            uint32_t he = 0, hc = 0;
            bool replay = false;
            PROF_T0(pw);
            bool any = world_hit<kKind, kF>(S, P.prune_delta, ray, g, k, t, he, hc, stk, mode, replay);
            PROF_ADD(kPrWorld, pw);
            if (kKind == 0 && replay) {  // hand the sample to the reference kernel
                unsigned idx = atomicAdd(&ctr->replay_count, 1u);
                if (idx < kReplayCap) replay_publish(replay_list, idx, g.pixel, g.sample - Q.sample0);
                has = false;
            } else if (finish_segment<kF>(S, P, Q, k, sbuf, any, he, hc, t, ray, L, T, depth, g, slot, g.sample - Q.sample0)) {
                has = false;
                nseg += P.max_depth - depth + (depth != 0u ? 1u : 0u);
            }
        }
    }
    if (kKind == 2) {
        __syncthreads();
        if (lane < 4u * S.hrpp_npred) atomicAdd(&S.hrpp_stats[lane], (unsigned long long)S.hrpp_cnt[lane]);
    }
    if (seg_counter) {
        unsigned long long v = (unsigned long long)nseg;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0u) {
            atomicAdd(seg_counter, v);
            if (kKind == 0 || stream_grid) atomicAdd(&ctr->fast_segments, v);
        }
    }
    if (kKind == 0 && lane == 0u) {  // count the wave out for the streaming replay pass
        __threadfence();  // (release: its replay-list entries and replay_count increments first)
        atomicAdd(&ctr->fast_done, 1u);
    }
    PROF_FLUSH();
#ifdef RT_PROFILE_REGIONS
    if (kKind == 0 && lane == 0u && tp_acc && tp_bucket < kTpBuckets) atomicAdd(&g_tp_hist[tp_bucket], tp_acc);
    if (stream_grid && lane == 0u) role_event(0xfffffffeu);
    if (kKind == 0 && lane == 0u && blockIdx.x < kProfWaves) {
        g_wave_t[2u * blockIdx.x] = wave_t0;
        g_wave_t[2u * blockIdx.x + 1u] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// color_accumulator += ray_color(...) in sample order, then / spp (renderer.rs:140-147).
// Chunks continue the same running sum held in `out`.
__global__ __launch_bounds__(256) void resolve_samples(const float* __restrict__ sbuf, float* __restrict__ out,
                                                        DevParams P, ChunkParams Q, int first, int last) {
    // one thread per sample-buffer slot (block-major: 64 consecutive slots are one 8x8 block,
    // so every plane is read in full, coalesced lines)
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= Q.nslots) return;
    const uint32_t blk = P.shard_index + (t >> 6) * P.shard_count, pib = t & 63u;
    const uint32_t by = blk / P.blocks_x, bx = blk - by * P.blocks_x;
    const uint32_t x = bx * 8u + (pib & 7u), y = by * 8u + (pib >> 3);
    if (x >= P.width || y >= P.height) return;
    float* o = out + ((size_t)y * P.width + x) * 3u;
    V acc = first ? mk(0.0f, 0.0f, 0.0f) : mk(o[0], o[1], o[2]);
    const float* src = sbuf + (size_t)t * 3u;
    const size_t plane = (size_t)Q.nslots * 3u;
    for (uint32_t s = 0; s < Q.samples; ++s) {
        acc = acc + mk(src[0], src[1], src[2]);
        src += plane;
    }
    if (last) acc = divs(acc, (float)P.spp_div);
    o[0] = acc.x;
    o[1] = acc.y;
    o[2] = acc.z;
}

// Device numeric self-check (rt_device_numeric_eval).
__global__ void numeric_eval(int op, const double* a, const double* b, double* out, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = a[i], y = b ? b[i] : 0.0;
    double r = 0.0;
    switch (op) {
        case 0: r = __builtin_sqrt(x); break;
        case 1: r = (double)__builtin_sqrtf((float)x); break;
        case 2: r = (double)((float)x / (float)y); break;
        case 3: r = (double)rt_sinf((float)x); break;
        case 4: r = (double)rt_acosf((float)x); break;
        case 5: r = (double)rt_atan2f((float)x, (float)y); break;
        case 6: r = (double)rt_logf((float)x); break;
        case 7: r = x / y; break;
        case 8: r = (double)hrpp_map_float((float)x); break;
        default: r = 0.0; break;
    }
    out[i] = r;
}

// Device known-answer evaluation (rt_device_kat): the kernel's own primitives on
// caller-supplied inputs, for the reference's unit tests run on the GPU.
__global__ void kat_eval(int op, const float* __restrict__ in, float* __restrict__ out, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float r0 = 0.0f, r1 = 0.0f;
    if (op == 0 || op == 1) {  // Aabb::hit (aabb.rs:28-41): min, max, origin, direction, t_min, t_max
        const float* a = in + 14u * i;
        Ray r;
        r.o = mk(a[6], a[7], a[8]);
        r.d = mk(a[9], a[10], a[11]);
        r.time = 0.0f;
        const V inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
        if (op == 0) {  // the reference-exact slab test (bvh_hit_reference, the BVH root test)
            float te = 0.0f;
            r0 = slab(a[0], a[1], a[2], a[3], a[4], a[5], r, inv, a[12], a[13], te) ? 1.0f : 0.0f;
            r1 = te;
        } else {  // the packed four-child test of the fast kernel, box in slot 0, empty slots 1-3
            const float E = kInf;
            f4 mnx{a[0], E, E, E}, mny{a[1], E, E, E}, mnz{a[2], E, E, E};
            f4 mxx{a[3], -E, -E, -E}, mxy{a[4], -E, -E, -E}, mxz{a[5], -E, -E, -E};
            float key[4];  // rows ordered by the direction signs, as bvh_run loads them
            child_keys4_nf(inv.x < 0.0f ? mxx : mnx, inv.y < 0.0f ? mxy : mny, inv.z < 0.0f ? mxz : mnz,
                           inv.x < 0.0f ? mnx : mxx, inv.y < 0.0f ? mny : mxy, inv.z < 0.0f ? mnz : mxz, r, inv,
                           a[12], a[13], kInf, 0.0f, key);
            r0 = key[0] != kInf ? 1.0f : 0.0f;
            r1 = key[0];
        }
    } else if (op == 2) {  // Sphere::get_uv (sphere.rs:41-46)
        const float* a = in + 3u * i;
        sphere_uv(mk(a[0], a[1], a[2]), r0, r1);
    } else if (op == 4) {  // a cube side's (k - o) / d the way a BVH cube leaf forms it, and the division
        const float kk = in[3u * i], o = in[3u * i + 1u], d = in[3u * i + 2u];
        const auto zero = [](float v) { return (__float_as_uint(v) & 0x7fffffffu) == 0u; };
        const bool gate = (__float_as_uint(kk) == 0u || rcp_range(kk)) && (zero(o) || rcp_range(o)) && rcp_range(d);
        r0 = gate ? rcp_quotient(kk, o, d, 1.0f / d) : (kk - o) / d;
        r1 = (kk - o) / d;
    } else if (op == 3) {  // Sphere::hit's root (sphere.rs:49-103): center, radius, origin, direction, t_min, t_max
        const float* a = in + 12u * i;
        Ray r;
        r.o = mk(a[4], a[5], a[6]);
        r.d = mk(a[7], a[8], a[9]);
        r.time = 0.0f;
        float t = 0.0f;
        r0 = sphere_t(f4{a[0], a[1], a[2], a[3]}, to_d(r), a[10], a[11], t) ? 1.0f : 0.0f;
        r1 = t;
    }
    out[2u * i] = r0;
    out[2u * i + 1u] = r1;
}

}  // namespace

#if defined(RT_INSTANCES_TU) && RT_INSTANCES_TU == 1
// kernel_mc.hip: this translation unit holds only the 4-wave instances of the
// BVH-only and the sphere-run presets, built with the memory-clause scheduler.
void* rt_mc_trace_instance(uint32_t preset) {
    if (preset == kFBvh) return reinterpret_cast<void*>(trace_samples<0, 4, kFBvh>);
    if (preset == (kFBvh | kFMarble)) return reinterpret_cast<void*>(trace_samples<0, 4, kFBvh | kFMarble>);
    if (preset == kFRuns) return reinterpret_cast<void*>(trace_samples<0, 4, kFRuns>);
    return nullptr;
}
#elif defined(RT_INSTANCES_TU) && RT_INSTANCES_TU == 2
// kernel_flat.hip: the flat-list preset (no BVH, no long sphere runs: C5), camera read from memory.
void* rt_flat_trace_instance(int waves) {
    return waves == 4 ? reinterpret_cast<void*>(trace_samples<0, 4, 0u>) : reinterpret_cast<void*>(trace_samples<0, 3, 0u>);
}
#else
#ifdef RT_SPLIT_MC
void* rt_mc_trace_instance(uint32_t preset);  // kernel_mc.hip
void* rt_flat_trace_instance(int waves);      // kernel_flat.hip
#endif

// ===========================================================================
// C ABI (device half)
// ===========================================================================
namespace {
// Table occupancy per predictor: out[2 p] = keys, out[2 p + 1] = stored leaf nodes.
__global__ __launch_bounds__(256) void hrpp_count(const rtdev::HrppSlot* __restrict__ tab, uint32_t bits, uint32_t np,
                                                  unsigned long long* __restrict__ out) {
    const uint64_t per = 1ull << bits;
    for (uint32_t p = 0; p < np; ++p) {
        unsigned long long keys = 0, ids = 0;
        for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < per; i += (uint64_t)gridDim.x * 256u) {
            const rtdev::HrppSlot& sl = tab[(uint64_t)p * per + i];
            if (sl.key == ~0ull) continue;
            keys += 1;
            for (uint32_t j = 0; j < rtdev::kHrppIds; ++j) ids += sl.ids[j] != 0xffffffffu ? 1u : 0u;
        }
        for (int off = 32; off > 0; off >>= 1) {
            keys += __shfl_xor(keys, off);
            ids += __shfl_xor(ids, off);
        }
        if ((threadIdx.x & 63u) == 0u) {
            atomicAdd(&out[2 * p], keys);
            atomicAdd(&out[2 * p + 1], ids);
        }
    }
}
// The launch's camera into device memory (RT_CAMMEM instances read it there). The value travels
// as a kernel argument, captured when the launch is enqueued, so no host buffer has to outlive
// the call (a hipMemcpyAsync from the caller's stack would rely on the runtime staging pageable
// copies before it returns).
__global__ void store_camera(DevCamera c, DevCamera* __restrict__ dst) {
    constexpr uint32_t kWords = sizeof(DevCamera) / sizeof(uint32_t);
    static_assert(sizeof(DevCamera) % sizeof(uint32_t) == 0, "DevCamera is whole words");
    const uint32_t i = threadIdx.x;
    if (i < kWords) {
        uint32_t w;
        __builtin_memcpy(&w, reinterpret_cast<const char*>(&c) + 4u * i, 4u);
        reinterpret_cast<uint32_t*>(dst)[i] = w;
    }
}
}  // namespace

struct rt_scene {
    int device = 0;
    void* pool = nullptr;
    uint64_t pool_bytes = 0;
    DevScene dev{};
    uint64_t counts[10] = {};
    // render workspace (sample buffer, counters, replay list), grown on demand; one render
    // at a time per scene handle
    float* sbuf = nullptr;
    uint64_t sbuf_bytes = 0;
    TraceCounters* counter = nullptr;
    uint32_t stack_ref = 1;  // LDS stack entries per lane of trace_samples<1, 2> (dev.stack_depth: <0>)
    int grid = 0, grid_ref = 0;  // resident waves of trace_samples<0> / <1>
    int fast_waves = 0;          // 3 or 4: the trace_samples<0, kWaves, kF> instance this scene launches
    uint32_t features = kFAll;   // kF bits the scene needs (BVHs, triangles, long sphere runs, deep stacks)
    uint32_t* stack_spill = nullptr;  // kFDeep: HBM stack entries past kStackLdsMax, grid x spill_depth x 64 x 2 words
    ReplayItem* replay = nullptr;  // kReplayCap entries, kReplayFree between chunks
    // the streaming replay pass runs on `aux`, forked from and joined back into the launch's stream
    hipStream_t aux = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    float coord_bound = 0.0f;
    // HRPP experiment: tables (allocated at the first RT_FLAG_HRPP render) and counters
    rtdev::HrppSlot* hrpp_tab = nullptr;
    uint64_t hrpp_tab_bytes = 0;
    uint32_t hrpp_bits = 0;
    unsigned long long* hrpp_stats = nullptr;  // kHrppMaxPredictors x 4
    // HIP events bracketing every trace launch (rt_scene_trace_time)
    static constexpr int kEvents = 256;
    hipEvent_t ev[kEvents][2] = {};
    int ev_count = 0;
    bool ev_overflow = false;
    // Launches on one handle share the workspace above: the host state is guarded by
    // `mu`, and each launch's stream waits for the previous launch's `done` event.
    std::mutex mu;
    hipEvent_t done = nullptr;
};

namespace {

int hip_fail(hipError_t e, const char* what) {
    return rthost::set_error(RT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {  // restores the caller's current device (e.g. torch's)
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// The fast-kernel instance for a scene: the first feature preset that covers the
// scene's features (flat lists; flat lists with long sphere runs; BVHs without
// triangles; BVHs with triangles and deep stacks; everything).
using TraceKernel = void (*)(DevScene, DevCamera, DevParams, ChunkParams, float*, TraceCounters*, ReplayItem*, uint32_t,
                             unsigned long long*);
// With RT_SPLIT_MC (the product build) the 4-wave BVH-only and sphere-run instances
// come from kernel_mc.hip, compiled with the memory-clause scheduling strategy:
// measured on the same box it is 1.3% faster on C3 and 1.2% on C2 but 1-2% slower
// on the other presets (C4, C5), and a scheduling strategy is a per-file flag.
// The flat-list instances come from kernel_flat.hip, which reads the camera from its device
// copy (RT_CAMMEM).
template <int kWaves, uint32_t kF>
TraceKernel preset_instance() {
#ifdef RT_SPLIT_MC
    if constexpr (kWaves == 4 && (kF == kFBvh || kF == (kFBvh | kFMarble) || kF == kFRuns))
        return reinterpret_cast<TraceKernel>(rt_mc_trace_instance(kF));
    else if constexpr (kF == 0u)
        return reinterpret_cast<TraceKernel>(rt_flat_trace_instance(kWaves));
    else
#endif
        return trace_samples<0, kWaves, kF>;
}
template <int kWaves>
TraceKernel fast_instance(uint32_t features) {
    switch (preset_of(features)) {  // (the presets preset_of names)
        case 0u: return preset_instance<kWaves, 0u>();
        case kFRuns: return preset_instance<kWaves, kFRuns>();
        case kFBvh: return preset_instance<kWaves, kFBvh>();
        case kFBvh | kFMarble: return preset_instance<kWaves, kFBvh | kFMarble>();
        case kFBvh | kFTri | kFDeep | kFSusp:
            return preset_instance<kWaves, kFBvh | kFTri | kFDeep | kFSusp>();
        default: return preset_instance<kWaves, kFAll>();
    }
}
TraceKernel fast_instance(int waves, uint32_t features) {
    return waves == 4 ? fast_instance<4>(features) : fast_instance<3>(features);
}

// rt_set_option's process-wide diagnostic switches (include/rt.h rt_option).
std::atomic<int64_t> g_opt[RT_OPT_COUNT] = {{0}, {0}, {0}, {0}, {-1}, {0}, {0}, {0}, {0}};
int64_t opt(int o) { return g_opt[o].load(std::memory_order_relaxed); }

int check_device(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return rthost::set_error(RT_ERR_NO_DEVICE, "no HIP device visible (the device path has no CPU fallback)");
    if (device < 0 || device >= n) return rthost::set_error(RT_ERR_INVALID, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return rthost::set_error(RT_ERR_NO_DEVICE, "device query failed");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return rthost::set_error(RT_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName +
                                                       "; this build targets gfx950 (MI355X) only");
    return RT_OK;
}

int check_params(const rt_render_params* p) {
    if (!p) return rthost::set_error(RT_ERR_INVALID, "params is NULL");
    if (p->width == 0 || p->height == 0) return rthost::set_error(RT_ERR_INVALID, "empty image");
    if (p->samples_per_pixel == 0) return rthost::set_error(RT_ERR_INVALID, "samples_per_pixel must be > 0");
    if (p->tile_width == 0 || p->tile_height == 0) return rthost::set_error(RT_ERR_INVALID, "tile size must be >= 1");
    if (p->shard_count > 1 && p->shard_index >= p->shard_count)
        return rthost::set_error(RT_ERR_INVALID, "shard_index >= shard_count");
    if ((uint64_t)p->width * p->height > 0x7fffffffull) return rthost::set_error(RT_ERR_INVALID, "image too large");
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_device_count(int* count) {
    rthost::clear_error();
    if (!count) return rthost::set_error(RT_ERR_INVALID, "count is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return RT_OK;
}

int rt_scene_upload(const rt_scene_desc* desc, int device, rt_scene_handle* out) {
    rthost::clear_error();
    if (!out) return rthost::set_error(RT_ERR_INVALID, "out is NULL");
    *out = nullptr;
    rthost::HostScene hs;
    std::string err;
    // Large BVHs are ordered on the target device (bvh_build.hip); RT_OPT_BVH_BUILD overrides.
    const int64_t mode = opt(RT_OPT_BVH_BUILD);
    int dev = device;
    rthost::BvhOrderer orderer{16384u, rthost::device_bvh_order, &dev};
    if (mode == 2) orderer.min_items = 1u;
    const bool host_only = mode == 1;
    int rc = rthost::lower_scene(desc, &hs, &err, host_only ? nullptr : &orderer, (int)opt(RT_OPT_BVH_SHAPE));
    if (rc) return rthost::set_error(rc, err);
    if (hs.max_stack > 96 || hs.max_stack_ref > 96)
        return rthost::set_error(RT_ERR_UNSUPPORTED, "BVH too deep for the LDS traversal stack");
    if ((rc = check_device(device))) return rc;
    if (hs.num_predictors > rtdev::kHrppMaxPredictors)
        return rthost::set_error(RT_ERR_UNSUPPORTED, "more than 8 Bvh::with_predictor BVHs");
    struct Part {
        const void* src;
        uint64_t bytes;
        uint64_t off;
    };
    std::vector<Part> parts = {
        {hs.entries.data(), hs.entries.size() * sizeof(DevEntry), 0},
        {hs.sph.data(), hs.sph.size() * sizeof(f4), 0},
        {hs.sph_mat.data(), hs.sph_mat.size() * sizeof(uint32_t), 0},
        {hs.msph.data(), hs.msph.size() * sizeof(f4), 0},
        {hs.rect.data(), hs.rect.size() * sizeof(f4), 0},
        {hs.tri.data(), hs.tri.size() * sizeof(f4), 0},
        {hs.nodes.data(), hs.nodes.size() * sizeof(f4), 0},
        {hs.mats.data(), hs.mats.size() * sizeof(DevMaterial), 0},
        {hs.texs.data(), hs.texs.size() * sizeof(DevTexture), 0},
        {hs.perm.data(), hs.perm.size(), 0},
        {hs.texels.data(), hs.texels.size(), 0},
        {hs.nodes2.data(), hs.nodes2.size() * sizeof(f4), 0},
        {hs.hrpp_keys.data(), hs.hrpp_keys.size() * sizeof(uint64_t), 0},
        {hs.hrpp_vals.data(), hs.hrpp_vals.size() * sizeof(uint32_t), 0},
    };
    uint64_t total = 0;
    for (auto& p : parts) {
        p.off = total;
        total += (p.bytes + 255u) & ~255ull;
    }
    if (total == 0) total = 256;
    rt_scene* s = new (std::nothrow) rt_scene();
    if (!s) return rthost::set_error(RT_ERR_OOM, "host allocation failed");
    s->device = device;
    {
        DeviceGuard g(device);
        hipError_t e = hipMalloc(&s->pool, total);
        if (e != hipSuccess) {
            delete s;
            return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc scene: ") + hipGetErrorString(e));
        }
        std::vector<uint8_t> staging(total, 0);
        for (auto& p : parts)
            if (p.bytes) memcpy(staging.data() + p.off, p.src, p.bytes);
        e = hipMemcpy(s->pool, staging.data(), total, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(s->pool);
            delete s;
            return hip_fail(e, "hipMemcpy scene");
        }
    }
    uint8_t* base = (uint8_t*)s->pool;
    s->pool_bytes = total;
    DevScene& d = s->dev;
    d.entries = (const DevEntry*)(base + parts[0].off);
    d.sph = (const f4*)(base + parts[1].off);
    d.sph_mat = (const uint32_t*)(base + parts[2].off);
    d.msph = (const f4*)(base + parts[3].off);
    d.rect = (const f4*)(base + parts[4].off);
    d.tri = (const f4*)(base + parts[5].off);
    d.nodes = (const f4*)(base + parts[6].off);
    d.mats = (const DevMaterial*)(base + parts[7].off);
    d.texs = (const DevTexture*)(base + parts[8].off);
    d.num_mats = (uint32_t)hs.mats.size();
    d.num_texs = (uint32_t)hs.texs.size();
    d.mt_lds = 0u;  // set per launch (the flat-list preset)
    d.perm = base + parts[9].off;
    d.texels = base + parts[10].off;
    d.nodes2 = (const f4*)(base + parts[11].off);
    d.num_nodes = (uint32_t)(hs.nodes.size() / rtdev::kBvhNodeF4);
    d.num_nodes2 = (uint32_t)(hs.nodes2.size() / 4);
    d.num_top = hs.num_top;
    d.num_entries = (uint32_t)hs.entries.size();
    d.stack_depth = hs.max_stack;
#ifdef RT_LEAF_AUDIT
    // the audit replays every fast traversal with the BVH2 recursion on the same stack
    d.stack_depth = std::max(hs.max_stack, hs.max_stack_ref);
#endif
    s->stack_ref = hs.max_stack_ref;
    d.perm_bytes = (uint32_t)hs.perm.size();
    d.hrpp_tab = nullptr;  // set per RT_FLAG_HRPP launch
    d.hrpp_keys = (const unsigned long long*)(base + parts[12].off);
    d.hrpp_vals = (const uint32_t*)(base + parts[13].off);
    d.hrpp_nkeys = (uint32_t)hs.hrpp_keys.size();
    d.hrpp_npred = hs.num_predictors;
    s->coord_bound = hs.coord_bound;
    d.rect_rcp_ok = 1u;  // div_rn_safe's scene half: rect / cube-side coordinates +0 or in [2^-20, 2^20]
    for (size_t i = 0; i + 1 < hs.rect.size(); i += 2) {  // (k, a0, a1, b0) (b1, axis, mat, 0)
        const rtdev::f4 r0 = hs.rect[i], r1 = hs.rect[i + 1];
        for (float c : {r0.x, r0.y, r0.z, r0.w, r1.x}) {
            uint32_t b;
            memcpy(&b, &c, 4);
            const float a = std::fabs(c);
            if (!(b == 0u || (a >= 0x1p-20f && a <= 0x1p20f))) d.rect_rcp_ok = 0u;
        }
    }
    d.mb_entry = ~0u;  // the medium-first bound's entry (medium_first_estimate)
    for (uint32_t e = 0; e < hs.num_top; ++e) {
        const rtdev::DevEntry& E = hs.entries[e];
        if (E.kind == rtdev::kEntMedium) {
            const rtdev::DevEntry& B = hs.entries[E.payload];
            if (B.kind == rtdev::kEntGeom && rtdev::leaf_type(B.payload) == rtdev::kLeafSphere) d.mb_entry = e;
            break;
        }
        bool ok = E.kind == rtdev::kEntSphereRun || E.kind == rtdev::kEntRectRun;
        if (E.kind == rtdev::kEntGeom) ok = rtdev::leaf_type(E.payload) != rtdev::kLeafTri;
        if (E.kind == rtdev::kEntBvh) {
            uint32_t flag;
            memcpy(&flag, &hs.nodes[(size_t)E.payload * rtdev::kBvhNodeF4 + 7].w, 4);
            ok = (flag & rtdev::kBvhPrunable) != 0u;
            for (uint32_t i = 0; i < E.ntf && i < (uint32_t)rtdev::kMaxTransforms; ++i) ok = ok && E.tf[i].w == 0.0f;
        }
        if (!ok) break;
    }
    s->features = (hs.tri.empty() ? 0u : kFTri) | (hs.bvh_rect_msph ? kFLeafRM : 0u);
    for (const rtdev::DevTexture& t : hs.texs)
        if (t.kind == rtdev::kTexMarble) s->features |= kFMarble;
#ifndef RT_LEAF_AUDIT  // (the audit build replays traversals on the same LDS stack: no spill area)
    {  // deep BVHs: the LDS stack keeps kStackLdsMax entries, HBM the rest
        uint32_t cap = kStackLdsMax;
        if (const int64_t v = opt(RT_OPT_STACK_LDS))  // diagnostics / tests: a smaller LDS part (>= 1)
            cap = std::min(cap, (uint32_t)v);
        if (hs.max_stack > cap) {
            s->features |= kFDeep;
            d.stack_depth = cap;
            d.spill_depth = hs.max_stack - cap;
        }
    }
#endif
    for (const rtdev::DevEntry& e : hs.entries) {  // top-level entries and medium boundaries
        if (e.kind == rtdev::kEntBvh) s->features |= kFBvh;
        if (e.kind == rtdev::kEntSphereRun && e.pad[0] >= kRunPretestMin) s->features |= kFRuns;
    }
    uint64_t c[10] = {hs.entries.size(), hs.sph.size(), hs.msph.size() / 3, hs.rect.size() / 2, hs.tri.size() / 3,
                      hs.nodes.size() / rtdev::kBvhNodeF4, hs.mats.size(), hs.texs.size(), hs.max_bvh_depth, total};
    memcpy(s->counts, c, sizeof c);
    *out = s;
    return RT_OK;
}

int rt_scene_free(rt_scene_handle s) {
    rthost::clear_error();
    if (!s) return RT_OK;
    {
        DeviceGuard g(s->device);
#ifdef RT_PROFILE_REGIONS
        static unsigned long long hc[kProfCopies * kProfWords];
        unsigned long long h[kProfWords] = {};
        if (hipDeviceSynchronize() == hipSuccess && hipMemcpyFromSymbol(hc, HIP_SYMBOL(g_prof), sizeof hc) == hipSuccess) {
            for (uint32_t c = 0; c < kProfCopies; ++c)
                for (uint32_t i = 0; i < kProfWords; ++i) h[i] += hc[c * kProfWords + i];
            fprintf(stderr, "{\"rt_profile\": [");
            for (uint32_t i = 0; i < 3u * kPrCount; ++i) fprintf(stderr, "%s%llu", i ? "," : "", h[i]);
            fprintf(stderr, "]}\n");
        }
        {
            const unsigned long long* th = h + 3u * kPrCount;
            fprintf(stderr, "{\"trips_hist\": [%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu], \"wave_max_hist\": "
                            "[%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu]}\n",
                    th[0], th[1], th[2], th[3], th[4], th[5], th[6], th[7], th[8], th[9], th[10], th[11], th[12],
                    th[13], th[14], th[15]);
        }
        {
            static unsigned long long wt[2 * kProfWaves];
            if (hipMemcpyFromSymbol(wt, HIP_SYMBOL(g_wave_t), sizeof wt) == hipSuccess) {
                std::vector<unsigned long long> st, en;
                for (uint32_t i = 0; i < kProfWaves; ++i)
                    if (wt[2 * i + 1]) {
                        st.push_back(wt[2 * i]);
                        en.push_back(wt[2 * i + 1]);
                    }
                if (!st.empty()) {
                    std::sort(st.begin(), st.end());
                    std::sort(en.begin(), en.end());
                    const unsigned long long t0 = st.front();
                    auto q = [&](const std::vector<unsigned long long>& v, double f) {
                        return (double)(v[(size_t)(f * (double)(v.size() - 1))] - t0) / 100.0;  // 100 MHz -> us
                    };
                    fprintf(stderr, "{\"wave_times_us\": {\"waves\": %zu, \"start\": [%.1f, %.1f, %.1f], "
                                    "\"end\": [%.1f, %.1f, %.1f, %.1f, %.1f]}}\n",
                            st.size(), q(st, 0.5), q(st, 0.99), q(st, 1.0), q(en, 0.0), q(en, 0.1), q(en, 0.5),
                            q(en, 0.9), q(en, 1.0));
                }
            }
            static unsigned long long rv[2 * kRoleEvents];
            unsigned rn = 0;
            if (hipMemcpyFromSymbol(&rn, HIP_SYMBOL(g_role_n), sizeof rn) == hipSuccess && rn &&
                hipMemcpyFromSymbol(rv, HIP_SYMBOL(g_role_ev), sizeof rv) == hipSuccess) {
                unsigned long long t0 = ~0ull;
                for (uint32_t i = 0; i < kProfWaves; ++i)
                    if (wt[2 * i + 1] && wt[2 * i] < t0) t0 = wt[2 * i];
                fprintf(stderr, "{\"role_events_us\": [");
                for (unsigned i = 0; i < rn && i < kRoleEvents; ++i)
                    fprintf(stderr, "%s[%.1f, %lld]", i ? "," : "", ((double)rv[2 * i] - (double)t0) / 100.0,
                            rv[2 * i + 1] >= 0xfffffffeull ? -(long long)(rv[2 * i + 1] - 0xfffffffdull) : (long long)rv[2 * i + 1]);
                fprintf(stderr, "]}\n");
            }
            static unsigned long long tp[kTpBuckets];
            if (hipMemcpyFromSymbol(tp, HIP_SYMBOL(g_tp_hist), sizeof tp) == hipSuccess) {
                uint32_t n = kTpBuckets;
                while (n > 0u && tp[n - 1u] == 0u) --n;
                fprintf(stderr, "{\"tp_gseg_per_s\": {\"bucket_us\": %u, \"rate\": [", kTpTicks / 100u);
                for (uint32_t i = 0; i < n; ++i)  // segments per bucket -> G segments / s
                    fprintf(stderr, "%s%.3f", i ? "," : "", (double)tp[i] / (kTpTicks * 10.0));
                fprintf(stderr, "]}}\n");
            }
        }
#endif
#ifdef RT_DEBUG_PIXEL
        {
            unsigned nd = 0;
            static uint32_t dv[8 * kDbgMax];
            if (hipMemcpyFromSymbol(&nd, HIP_SYMBOL(g_dbg_n), sizeof nd) == hipSuccess &&
                hipMemcpyFromSymbol(dv, HIP_SYMBOL(g_dbg), sizeof dv) == hipSuccess)
                for (unsigned i = 0; i < nd && i < kDbgMax; ++i)
                    fprintf(stderr, "DBG %u %08x %08x %08x %08x %08x %08x %08x\n", dv[8 * i], dv[8 * i + 1],
                            dv[8 * i + 2], dv[8 * i + 3], dv[8 * i + 4], dv[8 * i + 5], dv[8 * i + 6], dv[8 * i + 7]);
        }
#endif
#ifdef RT_LEAF_AUDIT
        unsigned na = 0;
        static LeafAudit au[kAuditMax];
        if (hipMemcpyFromSymbol(&na, HIP_SYMBOL(g_audit_count), sizeof na) == hipSuccess &&
            hipMemcpyFromSymbol(au, HIP_SYMBOL(g_audit), sizeof au) == hipSuccess) {
            fprintf(stderr, "{\"leaf_audit_count\": %u}\n", na);
            for (unsigned i = 0; i < na && i < kAuditMax; ++i)
                fprintf(stderr,
                        "{\"audit\": {\"o\": [%a, %a, %a], \"d\": [%a, %a, %a], \"tmin\": %a, \"closest\": %a, "
                        "\"t\": %a, \"box\": [%a, %a, %a, %a, %a, %a], \"delta\": %a, \"code\": %u, \"rank\": %u, "
                        "\"best_rank\": %u}}\n",
                        au[i].o[0], au[i].o[1], au[i].o[2], au[i].d[0], au[i].d[1], au[i].d[2], au[i].tmin,
                        au[i].closest, au[i].t, au[i].box[0], au[i].box[1], au[i].box[2], au[i].box[3], au[i].box[4],
                        au[i].box[5], au[i].delta, au[i].code, au[i].rank, au[i].best_rank);
        }
        static TravAudit ta[kAuditMax];
        if (hipMemcpyFromSymbol(&na, HIP_SYMBOL(g_trav_audit_count), sizeof na) == hipSuccess &&
            hipMemcpyFromSymbol(ta, HIP_SYMBOL(g_trav_audit), sizeof ta) == hipSuccess) {
            fprintf(stderr, "{\"trav_audit_count\": %u}\n", na);
            for (unsigned i = 0; i < na && i < kAuditMax; ++i)
                fprintf(stderr,
                        "{\"trav_audit\": {\"o\": [%a, %a, %a], \"d\": [%a, %a, %a], \"tmin\": %a, \"tmax\": %a, "
                        "\"fast_t\": %a, \"ref_t\": %a, \"fast_code\": %u, \"ref_code\": %u, \"root\": %u}}\n",
                        ta[i].o[0], ta[i].o[1], ta[i].o[2], ta[i].d[0], ta[i].d[1], ta[i].d[2], ta[i].tmin, ta[i].tmax,
                        ta[i].fast_t, ta[i].ref_t, ta[i].fast_code, ta[i].ref_code, ta[i].root);
        }
        if (hipMemcpyFromSymbol(&na, HIP_SYMBOL(g_bounds_audit_count), sizeof na) == hipSuccess)
            fprintf(stderr, "{\"bounds_audit_count\": %u}\n", na);
#endif
        if (s->done) (void)hipEventSynchronize(s->done);  // the last launch may still use the buffers below
        if (s->pool) (void)hipFree(s->pool);
        if (s->sbuf) (void)hipFree(s->sbuf);
        if (s->counter) (void)hipFree(s->counter);
        if (s->stack_spill) (void)hipFree(s->stack_spill);
        if (s->replay) (void)hipFree(s->replay);
        if (s->fork) (void)hipEventDestroy(s->fork);
        if (s->join) (void)hipEventDestroy(s->join);
        if (s->aux) (void)hipStreamDestroy(s->aux);
        if (s->hrpp_tab) (void)hipFree(s->hrpp_tab);
        if (s->hrpp_stats) (void)hipFree(s->hrpp_stats);
        for (int i = 0; i < rt_scene::kEvents; ++i)
            for (int j = 0; j < 2; ++j)
                if (s->ev[i][j]) (void)hipEventDestroy(s->ev[i][j]);
        if (s->done) (void)hipEventDestroy(s->done);
    }
    delete s;
    return RT_OK;
}

int rt_scene_hrpp_stats(rt_scene_handle s, uint64_t* out, uint32_t capacity, uint32_t* count) {
    rthost::clear_error();
    if (!s || !count) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    const uint32_t np = s->dev.hrpp_npred;
    *count = np;
    if (!out || capacity < 6u * np) return capacity == 0 ? RT_OK : rthost::set_error(RT_ERR_INVALID, "capacity < 6 per predictor");
    memset(out, 0, sizeof(uint64_t) * 6u * np);
    if (!s->hrpp_stats) return RT_OK;  // no RT_FLAG_HRPP render yet
    DeviceGuard g(s->device);
    unsigned long long h[4 * rtdev::kHrppMaxPredictors] = {};
    unsigned long long* d_tab_counts = nullptr;
    hipError_t e;
    if ((e = hipMalloc(&d_tab_counts, 16u * np)) != hipSuccess ||
        (e = hipMemset(d_tab_counts, 0, 16u * np)) != hipSuccess) {
        if (d_tab_counts) (void)hipFree(d_tab_counts);
        return hip_fail(e, "HRPP stats");
    }
    (void)hipGetLastError();
    if (s->hrpp_bits)
        hipLaunchKernelGGL(hrpp_count, dim3(1024), dim3(256), 0, nullptr, s->hrpp_tab, s->hrpp_bits, np, d_tab_counts);
    unsigned long long tc[2 * rtdev::kHrppMaxPredictors] = {};
    if ((e = hipGetLastError()) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess ||
        (e = hipMemcpy(h, s->hrpp_stats, 32u * np, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(tc, d_tab_counts, 16u * np, hipMemcpyDeviceToHost)) != hipSuccess) {
        (void)hipFree(d_tab_counts);
        return hip_fail(e, "HRPP stats");
    }
    (void)hipFree(d_tab_counts);
    for (uint32_t p = 0; p < np; ++p) {
        out[6 * p + 0] = h[4 * p + 0];
        out[6 * p + 1] = h[4 * p + 1];
        out[6 * p + 2] = h[4 * p + 2];
        out[6 * p + 3] = tc[2 * p + 0];
        out[6 * p + 4] = tc[2 * p + 1];
        out[6 * p + 5] = h[4 * p + 3];
    }
    return RT_OK;
}

int rt_scene_info(rt_scene_handle s, uint64_t counts[10]) {
    rthost::clear_error();
    if (!s || !counts) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    memcpy(counts, s->counts, sizeof s->counts);
    return RT_OK;
}

int rt_camera_new(const rt_camera_desc* args, rt_camera* out) {
    rthost::clear_error();
    if (!args || !out) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    std::string err;
    int rc = rthost::camera_new(args, out, &err);
    return rc ? rthost::set_error(rc, err) : RT_OK;
}

int rt_render_launch(rt_scene_handle s, const rt_camera_desc* camera, const rt_render_params* p, float* d_out,
                     unsigned long long* d_segments, void* stream) {
    rthost::clear_error();
    if (!camera) return rthost::set_error(RT_ERR_INVALID, "NULL camera");
    rt_camera cam;
    std::string err;
    int rc = rthost::camera_new(camera, &cam, &err);
    if (rc) return rthost::set_error(rc, err);
    return rt_render_launch_camera(s, &cam, p, d_out, d_segments, stream);
}

int rt_render_launch_camera(rt_scene_handle s, const rt_camera* camera, const rt_render_params* p, float* d_out,
                            unsigned long long* d_segments, void* stream) {
    rthost::clear_error();
    if (!s || !camera || !d_out) return rthost::set_error(RT_ERR_INVALID, "NULL scene/camera/output");
    int rc = check_params(p);
    if (rc) return rc;
    DevCamera cam;
    std::string err;
    if ((rc = rthost::camera_device(camera, &cam, &err))) return rthost::set_error(rc, err);
    DevParams dp;
    memset(&dp, 0, sizeof dp);
    dp.width = p->width;
    dp.height = p->height;
    dp.spp = p->samples_per_pixel;
    dp.max_depth = p->max_depth;
    dp.seed_lo = (uint32_t)p->seed;
    dp.seed_hi = (uint32_t)(p->seed >> 32);
    dp.sample_base = p->sample_base;
    dp.shard_count = p->shard_count > 1 ? p->shard_count : 1u;
    dp.shard_index = p->shard_count > 1 ? p->shard_index : 0u;
    dp.blocks_x = (p->width + 7u) / 8u;
    dp.num_blocks = dp.blocks_x * ((p->height + 7u) / 8u);
    dp.flags = p->flags;
    dp.spp_div = p->spp_total ? p->spp_total : p->samples_per_pixel;
    dp.tune = (uint32_t)opt(RT_OPT_TUNE) & ~kModeExact;  // diagnostic traversal switches (kMode* bits)
    dp.bg[0] = p->background[0];
    dp.bg[1] = p->background[1];
    dp.bg[2] = p->background[2];
    {
        // Pruning margin: every ray origin and hit point lies within R of the
        // origin of any BVH frame (camera + lens, scene coordinates, translations).
        double R = sqrt((double)cam.origin[0] * cam.origin[0] + (double)cam.origin[1] * cam.origin[1] +
                        (double)cam.origin[2] * cam.origin[2]) +
                   2.0 * (double)fabsf(cam.lens_radius) + 2.0 * (double)s->coord_bound;
        double delta = R * (1.0 / 1048576.0) * 1.01 + 1e-30;  // 2^-20 R
        dp.prune_delta = (float)delta;
        if (!(dp.prune_delta < 1e30f)) dp.flags |= RT_FLAG_EXACT_BVH;  // non-finite scene: no pruning
    }
    uint32_t nblk = dp.num_blocks > dp.shard_index ? (dp.num_blocks - dp.shard_index + dp.shard_count - 1u) / dp.shard_count : 0u;
#ifdef RT_PROFILE_REGIONS
    if (g_prof_rows[1] != 0xffffffffu && dp.shard_count == 1u) {  // rt_prof_rows: the band's blocks only
        const uint32_t rows = (dp.height + 7u) / 8u;
        const uint32_t r0 = std::min(g_prof_rows[0], rows), r1 = std::min(std::max(g_prof_rows[1], r0), rows);
        dp.shard_index = r0 * dp.blocks_x;  // block = shard_index + local block (shard_count 1)
        nblk = (r1 - r0) * dp.blocks_x;
    }
#endif
    if (nblk == 0) return RT_OK;
    DeviceGuard g(s->device);
    if (!g.ok) return rthost::set_error(RT_ERR_HIP, "hipSetDevice failed");
    // One render at a time per handle: host state under the lock, and on the device
    // this launch starts after the previous one (any stream) has finished.
    std::lock_guard<std::mutex> lock(s->mu);
    hipError_t e;
    if (!s->done && (e = hipEventCreateWithFlags(&s->done, hipEventDisableTiming)) != hipSuccess) {
        s->done = nullptr;
        return hip_fail(e, "hipEventCreate");
    }
    if ((e = hipStreamWaitEvent((hipStream_t)stream, s->done, 0)) != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
    // Sample buffer: chunks of whole sample ranges (the per-pixel sum stays in order).
    // the shard's 8x8 blocks, 64 slots each, block-major (dense for every shard: full cache lines)
    const uint64_t nslots = (uint64_t)nblk * 64u;
    const uint64_t per_sample = nslots * 3u * sizeof(float);
    // One launch per frame whenever HBM allows (each chunk ends with its own drain tail):
    // up to 40% of the free HBM, at least 8 GiB (C4's 1000-spp frame needs 24.9 GB, C5's 49.8 GB)
    uint64_t budget = 8192ull << 20;
    {
        size_t free_b = 0, total_b = 0;
        if (s->sbuf_bytes >= per_sample * p->samples_per_pixel) {
            budget = s->sbuf_bytes;  // the buffer already holds the whole frame
        } else if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            const uint64_t avail = (uint64_t)((double)(free_b + s->sbuf_bytes) * 0.4);
            if (avail > budget) budget = avail;
        }
    }
    if (const int64_t mb = opt(RT_OPT_SAMPLE_BUFFER_MB)) budget = (uint64_t)mb << 20;
    uint64_t max_s = budget / per_sample;
    if (max_s > 0x7fffffffull / nblk) max_s = 0x7fffffffull / nblk;  // (block, sample) units fit 31 bits
    if (max_s < 1) max_s = 1;
    uint32_t nchunks = (uint32_t)((p->samples_per_pixel + max_s - 1) / max_s);
    uint32_t chunk = (p->samples_per_pixel + nchunks - 1) / nchunks;
    uint64_t need = per_sample * chunk;
    if (s->sbuf_bytes < need) {
        if (s->sbuf) (void)hipFree(s->sbuf);
        s->sbuf = nullptr;
        s->sbuf_bytes = 0;
        if ((e = hipMalloc(&s->sbuf, need)) != hipSuccess)
            return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc sample buffer: ") + hipGetErrorString(e));
        s->sbuf_bytes = need;
    }
    if (!s->counter) {
        static_assert(sizeof(TraceCounters) <= kCamOffset, "counters then the camera copy");
        if ((e = hipMalloc(&s->counter, kCamOffset + sizeof(DevCamera))) != hipSuccess)
            return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc counter: ") + hipGetErrorString(e));
    }
    if (!s->replay) {
        if ((e = hipMalloc(&s->replay, sizeof(ReplayItem) * (size_t)kReplayCap)) != hipSuccess)
            return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc replay list: ") + hipGetErrorString(e));
        if ((e = hipMemsetAsync(s->replay, 0xff, sizeof(ReplayItem) * (size_t)kReplayCap, (hipStream_t)stream)) !=
            hipSuccess)  // every entry kReplayFree
            return hip_fail(e, "replay list reset");
    }
    if (!s->aux) {
        if ((e = hipStreamCreateWithFlags(&s->aux, hipStreamNonBlocking)) != hipSuccess) {
            s->aux = nullptr;
            return hip_fail(e, "hipStreamCreate (replay stream)");
        }
        if ((e = hipEventCreateWithFlags(&s->fork, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&s->join, hipEventDisableTiming)) != hipSuccess)
            return hip_fail(e, "hipEventCreate (replay stream)");
    }
    // The fast kernel's instance: four waves per SIMD when that raises its occupancy
    // over three (the Perlin tables then stay in L2, so the stack alone sets LDS) — except
    // for the BVH-only preset, whose 4-wave instance spills more than the extra wave buys
    // (same box, 3 vs 4 waves: C1 3.8 vs 4.1 ms; profiles/r05/experiments/waves_3v4_ab.log).
    // The triangle-BVH preset preferred 3 until round 5 (C4 at 50 spp 112.1 vs 121.4 ms in
    // round 2); with the rect runs and scalar entry reads its 4-wave instance became 2.2% faster
    // (1266 -> 1238 ms per frame), and round 6 returned to 3: within 1% of the 4-wave speed (C4 at
    // 50 spp 62.2 vs 61.7 ms) at an eighth of the HBM traffic (8.4 vs 63.8 GB per frame, the 4-wave
    // instance's ~40 spilled VGPRs; profiles/r06/experiments/sample_buffer_nt_and_waves_*). The
    // Marble, sphere-run and flat presets stay at 4 (C3 +12%, C2 +12%, C5 +10% over 3).
    const uint32_t preset_feats = s->features & ~kFDeep;
    const bool prefer3 = preset_feats == kFBvh || preset_feats == (kFBvh | kFTri);
    if (s->fast_waves == 0) {
        const size_t stack_lds = (size_t)s->dev.stack_depth * 128u * sizeof(uint32_t);
        const size_t perm3 = s->dev.perm_bytes != 0u && s->dev.perm_bytes <= kPermLdsMax ? s->dev.perm_bytes : 0u;
        int per3 = 0, per4 = 0;
        const TraceKernel k3 = fast_instance(3, s->features), k4 = fast_instance(4, s->features);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per3, k3, 64, stack_lds + perm3) != hipSuccess) per3 = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per4, k4, 64, stack_lds) != hipSuccess) per4 = 0;
        s->fast_waves = per4 > per3 && !(dp.tune & kModeW3) && (!prefer3 || (dp.tune & kModeW4)) ? 4 : 3;
    }
    if (s->fast_waves == 4) dp.tune |= kModeNoPermLds;
    // LDS per wave: the kernel's traversal stack, then the Perlin tables
    const size_t perm_lds =
        s->dev.perm_bytes != 0u && s->dev.perm_bytes <= kPermLdsMax && !(dp.tune & kModeNoPermLds) ? s->dev.perm_bytes : 0u;
    size_t lds = (size_t)s->dev.stack_depth * 128u * sizeof(uint32_t) + perm_lds;
    // the flat-list preset stages a small scene's materials and textures behind the stack (the fast
    // kernel's launch only: the reference and replay launches below reserve no LDS for them)
    const size_t mt_bytes = (size_t)(s->dev.num_mats + s->dev.num_texs) * 32u;
    const bool mt_stage = RT_MT_LDS && s->features == 0u && perm_lds == 0u && mt_bytes <= kMtLdsMax;
    s->dev.mt_lds = mt_stage ? (uint32_t)mt_bytes : 0u;
    if (mt_stage) lds += mt_bytes;
    DevScene dev_ref = s->dev;
    dev_ref.stack_depth = s->stack_ref;
    dev_ref.mt_lds = 0u;
    size_t lds_ref = (size_t)dev_ref.stack_depth * 128u * sizeof(uint32_t) + perm_lds;
    if ((dp.flags & RT_FLAG_HRPP) && s->dev.hrpp_npred) {  // the experiment: reference kernel + predictors
        dp.flags |= RT_FLAG_EXACT_BVH;
        const int64_t ob = opt(RT_OPT_HRPP_SLOT_BITS);
        const uint32_t bits = ob < 0 ? 22u : (uint32_t)ob;  // default 4 M slots (128 MiB) per predictor
        const uint64_t bytes = bits ? ((uint64_t)s->dev.hrpp_npred << bits) * sizeof(rtdev::HrppSlot) : 0u;
        if (s->hrpp_tab_bytes < bytes || !s->hrpp_stats) {
            if (s->hrpp_tab) (void)hipFree(s->hrpp_tab);
            s->hrpp_tab = nullptr;
            s->hrpp_tab_bytes = 0;
            if ((e = hipMalloc(&s->hrpp_tab, bytes ? bytes : sizeof(rtdev::HrppSlot))) != hipSuccess ||
                (!s->hrpp_stats && (e = hipMalloc(&s->hrpp_stats, 8u * 4u * rtdev::kHrppMaxPredictors)) != hipSuccess))
                return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc HRPP tables: ") + hipGetErrorString(e));
            s->hrpp_tab_bytes = bytes;
        }
        s->hrpp_bits = bits;
        if ((bytes && (e = hipMemsetAsync(s->hrpp_tab, 0xff, bytes, (hipStream_t)stream)) != hipSuccess) ||
            (e = hipMemsetAsync(s->hrpp_stats, 0, 8u * 4u * rtdev::kHrppMaxPredictors, (hipStream_t)stream)) !=
                hipSuccess)
            return hip_fail(e, "HRPP table reset");
        dev_ref.hrpp_tab = s->hrpp_tab;
        dev_ref.hrpp_stats = s->hrpp_stats;
        dev_ref.hrpp_bits = bits;
        lds_ref += 4u * rtdev::kHrppMaxPredictors * sizeof(uint32_t);
    }
    if (s->grid == 0) {
        int per_cu = 0, per_cu_ref = 0, cus = 0;
        const TraceKernel kf = fast_instance(s->fast_waves, s->features);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kf, 64, lds) != hipSuccess ||
            per_cu < 1)
            per_cu = 8;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_ref, trace_samples<1>, 64, lds_ref) != hipSuccess ||
            per_cu_ref < 1)
            per_cu_ref = 8;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device) != hipSuccess || cus < 1)
            cus = 256;
        s->grid = per_cu * cus;
        s->grid_ref = per_cu_ref * cus;
        if (s->features & kFDeep) {  // the deep-stack spill area: one slab per resident wave, then
            // kStreamWaves slabs for the streaming replay pass, which runs beside the fast kernel
            const size_t bytes = ((size_t)s->grid + kStreamWaves) * s->dev.spill_depth * 64u * 2u * sizeof(uint32_t);
            if ((e = hipMalloc(&s->stack_spill, bytes)) != hipSuccess) {
                s->grid = 0;
                return rthost::set_error(RT_ERR_OOM, std::string("hipMalloc stack spill: ") + hipGetErrorString(e));
            }
            s->dev.stack_spill = s->stack_spill;
        }
        if (opt(RT_OPT_LAUNCH_LOG))
            fprintf(stderr, "rt: trace_samples<0, %d, features 0x%x>: %d waves/CU (LDS %zu B/wave), reference kernel %d "
                    "waves/CU\n", s->fast_waves, s->features, per_cu, lds, per_cu_ref);
    }
    const bool exact = (dp.flags & RT_FLAG_EXACT_BVH) != 0u;
    hipStream_t st = (hipStream_t)stream;
    for (uint32_t c = 0; c < nchunks; ++c) {
        ChunkParams q;
        q.sample0 = p->sample_base + c * chunk;
        q.samples = c + 1 < nchunks ? chunk : p->samples_per_pixel - c * chunk;
        q.units = (uint32_t)(nblk * (uint64_t)q.samples);
        q.blocks = (uint32_t)nblk;
        q.group = batch_group(q.units, exact || dev_ref.hrpp_tab ? (uint32_t)s->grid_ref : (uint32_t)s->grid);
        if (const int64_t gr = opt(RT_OPT_GROUP)) q.group = (uint32_t)gr;  // diagnostics / A-B runs
        if (q.group > q.samples) q.group = q.samples;  // a batch crosses at most one block boundary
        q.guide = 2u;  // measured on C3 (63 and 500 spp): 2 beats 4, 8, 16 and 32 (tools/session_guide.sh)
        if (const int64_t gd = opt(RT_OPT_GUIDE)) q.guide = (uint32_t)gd;  // diagnostics / A-B runs
        q.nslots = (uint32_t)nslots;
        if ((e = hipMemsetAsync(s->counter, 0, sizeof(TraceCounters), st)) != hipSuccess)
            return hip_fail(e, "memset counters");
        // the launch's camera behind the counters: the flat-list instances (kernel_flat.hip, RT_CAMMEM)
        // read it from there at each new sample instead of keeping 21 camera words in SGPRs
        if (c == 0) {
            (void)hipGetLastError();  // sticky: drop an unrelated earlier error
            hipLaunchKernelGGL(store_camera, dim3(1), dim3(64), 0, st, cam,
                               reinterpret_cast<DevCamera*>(reinterpret_cast<char*>(s->counter) + kCamOffset));
            if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "camera store");
        }
        uint32_t grid = (uint32_t)s->grid, grid_ref = (uint32_t)s->grid_ref;
        if (grid > q.units) grid = q.units;
        if (grid_ref > q.units) grid_ref = q.units;
        q.fast_grid = grid;
        hipEvent_t* evp = nullptr;
        if (s->ev_count < rt_scene::kEvents) {
            evp = s->ev[s->ev_count];
            for (int j = 0; j < 2; ++j)
                if (!evp[j] && hipEventCreate(&evp[j]) != hipSuccess) evp = nullptr;
        } else {
            s->ev_overflow = true;
        }
        if (evp) (void)hipEventRecord(evp[0], st);
        (void)hipGetLastError();  // hipGetLastError is sticky: drop an unrelated earlier error
        if (dev_ref.hrpp_tab) {  // RT_FLAG_HRPP: the reference kernel with predictors
            hipLaunchKernelGGL(trace_samples<2>, dim3(grid_ref), dim3(64), lds_ref, st, dev_ref, cam, dp, q,
                               s->sbuf, s->counter, s->replay, 0u, d_segments);
        } else if (exact) {  // every BVH traversed by the literal replay of bvh.rs
            hipLaunchKernelGGL(trace_samples<1>, dim3(grid_ref), dim3(64), lds_ref, st, dev_ref, cam, dp, q,
                               s->sbuf, s->counter, s->replay, 0u, d_segments);
        } else {  // fast kernel, then the reference kernel on the samples it handed over
            const TraceKernel kf = fast_instance(s->fast_waves, s->features);
            // A deep-stack scene (C4) replays with trace_samples<3, 3, kFAll>: the streaming pass
            // spills into its own slabs behind the fast kernel's, the serialized remainder into the
            // fast kernel's, free by then (so that launch keeps to the fast kernel's grid).
            const bool deep = (s->features & kFDeep) != 0u;
            const bool kind3 = !(dp.tune & kModeReplayRef);
            // (not beside launches on other handles, RT_FLAG_FRAMES_IN_FLIGHT: its waves would be
            // dispatched in the other launch's drain, find this pool full and leave at once)
            const bool stream_rp = kind3 && !(dp.tune & kModeNoStream) && !(dp.flags & RT_FLAG_FRAMES_IN_FLIGHT);
            if (stream_rp && (e = hipEventRecord(s->fork, st)) != hipSuccess) return hip_fail(e, "replay stream fork");
            hipLaunchKernelGGL(kf, dim3(grid), dim3(64), lds, st, s->dev, cam, dp, q, s->sbuf, s->counter, s->replay,
                               0u, d_segments);
            if (kind3) {
                // the replay pass: fast traversal except for the rays that were handed over
                DevScene dev_rp = s->dev;
                dev_rp.stack_depth = std::max(s->dev.stack_depth, s->stack_ref);
                dev_rp.mt_lds = 0u;  // (only the fast kernel's launch stages them)
                const size_t lds_rp = (size_t)dev_rp.stack_depth * 128u * sizeof(uint32_t) + perm_lds;
                if (stream_rp) {  // streaming: takes the handed-over samples during the fast kernel's drain
                    // few waves: each polls the counters while it waits (3072 pollers slowed the
                    // drain they overlap by a third)
                    const uint32_t grid_st = std::min(grid_ref, kStreamWaves);
                    if ((e = hipStreamWaitEvent(s->aux, s->fork, 0)) != hipSuccess) return hip_fail(e, "replay stream wait");
                    if (deep) {
                        DevScene dev_st = dev_rp;
                        dev_st.stack_spill = s->stack_spill + (size_t)s->grid * s->dev.spill_depth * 64u * 2u;
                        hipLaunchKernelGGL((trace_samples<3, 3, kFAll>), dim3(grid_st), dim3(64), lds_rp, s->aux, dev_st,
                                           cam, dp, q, s->sbuf, s->counter, s->replay, 2u, d_segments);
                    } else {
                        hipLaunchKernelGGL((trace_samples<3, 3, kFAll & ~kFDeep>), dim3(grid_st), dim3(64), lds_rp,
                                           s->aux, dev_rp, cam, dp, q, s->sbuf, s->counter, s->replay, 2u, d_segments);
                    }
                    if ((e = hipEventRecord(s->join, s->aux)) != hipSuccess ||
                        (e = hipStreamWaitEvent(st, s->join, 0)) != hipSuccess)
                        return hip_fail(e, "replay stream join");
                }
                // serialized: whatever the streaming pass did not take (everything without it)
                if (deep)
                    hipLaunchKernelGGL((trace_samples<3, 3, kFAll>), dim3(std::min(grid_ref, grid)), dim3(64), lds_rp, st,
                                       dev_rp, cam, dp, q, s->sbuf, s->counter, s->replay, 1u, d_segments);
                else
                    hipLaunchKernelGGL((trace_samples<3, 3, kFAll & ~kFDeep>), dim3(grid_ref), dim3(64), lds_rp, st,
                                       dev_rp, cam, dp, q, s->sbuf, s->counter, s->replay, 1u, d_segments);
            } else {
                hipLaunchKernelGGL(trace_samples<1>, dim3(grid_ref), dim3(64), lds_ref, st, dev_ref, cam, dp, q,
                                   s->sbuf, s->counter, s->replay, 1u, d_segments);
            }
        }
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "trace_samples launch");
        if (opt(RT_OPT_LAUNCH_LOG)) {  // diagnostics: samples the fast kernel handed to the reference kernel
            TraceCounters h{};
            if (hipMemcpyAsync(&h, s->counter, sizeof h, hipMemcpyDeviceToHost, st) == hipSuccess &&
                hipStreamSynchronize(st) == hipSuccess)
                fprintf(stderr, "rt: chunk %u: %u samples replayed by the reference kernel\n", c, h.replay_count);
        }
        if (evp) {
            (void)hipEventRecord(evp[1], st);
            s->ev_count++;
        }
        hipLaunchKernelGGL(resolve_samples, dim3((uint32_t)((nslots + 255u) / 256u)), dim3(256), 0, st, s->sbuf, d_out, dp,
                           q, c == 0 && !(p->flags & RT_FLAG_ACCUMULATE) ? 1 : 0,
                           c + 1 == nchunks && !(p->flags & RT_FLAG_RAW_SUM) ? 1 : 0);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "resolve_samples launch");
    }
    if ((e = hipEventRecord(s->done, st)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    return RT_OK;
}

int rt_render(rt_scene_handle s, const rt_camera_desc* camera, const rt_render_params* p, float* host_out,
              rt_stats* stats) {
    rthost::clear_error();
    if (!camera) return rthost::set_error(RT_ERR_INVALID, "NULL camera");
    rt_camera cam;
    std::string err;
    int rc = rthost::camera_new(camera, &cam, &err);
    if (rc) return rthost::set_error(rc, err);
    return rt_render_camera(s, &cam, p, host_out, stats);
}

int rt_render_camera(rt_scene_handle s, const rt_camera* camera, const rt_render_params* p, float* host_out,
                     rt_stats* stats) {
    rthost::clear_error();
    if (!s || !camera || !host_out) return rthost::set_error(RT_ERR_INVALID, "NULL scene/camera/output");
    int rc = check_params(p);
    if (rc) return rc;
    DeviceGuard g(s->device);
    if (!g.ok) return rthost::set_error(RT_ERR_HIP, "hipSetDevice failed");
    size_t bytes = (size_t)p->width * p->height * 3u * sizeof(float);
    float* d_out = nullptr;
    unsigned long long* d_seg = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e;
    auto cleanup = [&]() {
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (st) (void)hipStreamDestroy(st);
        if (d_out) (void)hipFree(d_out);
        if (d_seg) (void)hipFree(d_seg);
    };
    if ((e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) != hipSuccess) { cleanup(); return hip_fail(e, "hipStreamCreate"); }
    if ((e = hipMalloc(&d_out, bytes)) != hipSuccess) { cleanup(); return rthost::set_error(RT_ERR_OOM, "hipMalloc image"); }
    if ((e = hipMalloc(&d_seg, sizeof(unsigned long long))) != hipSuccess) { cleanup(); return rthost::set_error(RT_ERR_OOM, "hipMalloc counter"); }
    if ((e = hipMemcpyAsync(d_out, host_out, bytes, hipMemcpyHostToDevice, st)) != hipSuccess) { cleanup(); return hip_fail(e, "H2D image"); }
    if ((e = hipMemsetAsync(d_seg, 0, sizeof(unsigned long long), st)) != hipSuccess) { cleanup(); return hip_fail(e, "memset"); }
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, st);
    rc = rt_render_launch_camera(s, camera, p, d_out, d_seg, st);
    if (rc) { cleanup(); return rc; }
    (void)hipEventRecord(e1, st);
    unsigned long long seg = 0;
    if ((e = hipMemcpyAsync(host_out, d_out, bytes, hipMemcpyDeviceToHost, st)) != hipSuccess) { cleanup(); return hip_fail(e, "D2H image"); }
    if ((e = hipMemcpyAsync(&seg, d_seg, sizeof seg, hipMemcpyDeviceToHost, st)) != hipSuccess) { cleanup(); return hip_fail(e, "D2H counter"); }
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return hip_fail(e, "render"); }
    if (stats) {
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        uint64_t pixels = 0;
        uint32_t sc = p->shard_count > 1 ? p->shard_count : 1u, si = p->shard_count > 1 ? p->shard_index : 0u;
        uint32_t bxn = (p->width + 7u) / 8u;
        for (uint32_t y = 0; y < p->height; ++y)
            for (uint32_t x = 0; x < p->width; ++x)
                if (((y / 8u) * bxn + x / 8u) % sc == si) pixels++;
        stats->segments = seg;
        stats->samples = pixels * p->samples_per_pixel;
        stats->kernel_ms = ms;
    }
    cleanup();
    return RT_OK;
}

int rt_render_multi(rt_scene_handle* scenes, uint32_t n, const rt_camera_desc* camera, const rt_render_params* p,
                    float* host_out, rt_stats* stats) {
    rthost::clear_error();
    if (!camera) return rthost::set_error(RT_ERR_INVALID, "NULL camera");
    rt_camera cam;
    std::string err;
    int rc = rthost::camera_new(camera, &cam, &err);
    if (rc) return rthost::set_error(rc, err);
    return rt_render_multi_camera(scenes, n, &cam, p, host_out, stats);
}

int rt_render_multi_camera(rt_scene_handle* scenes, uint32_t n, const rt_camera* camera, const rt_render_params* p,
                           float* host_out, rt_stats* stats) {
    rthost::clear_error();
    if (!scenes || n == 0 || !camera || !host_out) return rthost::set_error(RT_ERR_INVALID, "NULL argument or n == 0");
    int rc = check_params(p);
    if (rc) return rc;
    if (p->shard_count > 1) return rthost::set_error(RT_ERR_INVALID, "rt_render_multi shards the frame itself");
    for (uint32_t i = 0; i < n; ++i)
        if (!scenes[i]) return rthost::set_error(RT_ERR_INVALID, "NULL scene handle");
    const size_t floats = (size_t)p->width * p->height * 3u;
    struct Shard {
        int device = 0;
        hipStream_t st = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        float* d_out = nullptr;
        unsigned long long* d_seg = nullptr;
        unsigned long long seg = 0;
        std::vector<float> img;
    };
    std::vector<Shard> sh(n);
    auto cleanup = [&]() {
        for (Shard& x : sh) {
            DeviceGuard g(x.device);
            if (x.st) (void)hipStreamSynchronize(x.st);
            if (x.e0) (void)hipEventDestroy(x.e0);
            if (x.e1) (void)hipEventDestroy(x.e1);
            if (x.st) (void)hipStreamDestroy(x.st);
            if (x.d_out) (void)hipFree(x.d_out);
            if (x.d_seg) (void)hipFree(x.d_seg);
        }
    };
    hipError_t e;
    // launch every shard before waiting for any (devices run concurrently)
    for (uint32_t i = 0; i < n; ++i) {
        Shard& x = sh[i];
        x.device = scenes[i]->device;
        DeviceGuard g(x.device);
        if (!g.ok) { cleanup(); return rthost::set_error(RT_ERR_HIP, "hipSetDevice failed"); }
        if ((e = hipStreamCreateWithFlags(&x.st, hipStreamNonBlocking)) != hipSuccess) { cleanup(); return hip_fail(e, "hipStreamCreate"); }
        if ((e = hipMalloc(&x.d_out, floats * sizeof(float))) != hipSuccess ||
            (e = hipMalloc(&x.d_seg, sizeof(unsigned long long))) != hipSuccess) {
            cleanup();
            return rthost::set_error(RT_ERR_OOM, "hipMalloc shard image");
        }
        // RT_FLAG_ACCUMULATE continues the running sum the caller holds in host_out,
        // exactly like rt_render (which uploads it too)
        if (((p->flags & RT_FLAG_ACCUMULATE)
                 ? (e = hipMemcpyAsync(x.d_out, host_out, floats * sizeof(float), hipMemcpyHostToDevice, x.st))
                 : (e = hipMemsetAsync(x.d_out, 0, floats * sizeof(float), x.st))) != hipSuccess ||
            (e = hipMemsetAsync(x.d_seg, 0, sizeof(unsigned long long), x.st)) != hipSuccess) {
            cleanup();
            return hip_fail(e, "shard image init");
        }
        (void)hipEventCreate(&x.e0);
        (void)hipEventCreate(&x.e1);
        (void)hipEventRecord(x.e0, x.st);
        rt_render_params q = *p;
        q.shard_index = n > 1 ? i : 0u;
        q.shard_count = n > 1 ? n : 0u;
        if ((rc = rt_render_launch_camera(scenes[i], camera, &q, x.d_out, x.d_seg, x.st))) { cleanup(); return rc; }
        (void)hipEventRecord(x.e1, x.st);
        x.img.resize(floats);
        if ((e = hipMemcpyAsync(x.img.data(), x.d_out, floats * sizeof(float), hipMemcpyDeviceToHost, x.st)) != hipSuccess ||
            (e = hipMemcpyAsync(&x.seg, x.d_seg, sizeof x.seg, hipMemcpyDeviceToHost, x.st)) != hipSuccess) {
            cleanup();
            return hip_fail(e, "D2H shard");
        }
    }
    float ms_max = 0.0f;
    for (Shard& x : sh) {
        DeviceGuard g(x.device);
        if ((e = hipStreamSynchronize(x.st)) != hipSuccess) { cleanup(); return hip_fail(e, "render shard"); }
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, x.e0, x.e1);
        ms_max = ms > ms_max ? ms : ms_max;
    }
    // gather: every 8x8 block comes from the device that rendered it
    const uint32_t bxn = (p->width + 7u) / 8u;
    unsigned long long seg = 0;
    for (uint32_t y = 0; y < p->height; ++y)
        for (uint32_t x = 0; x < p->width; ++x) {
            const uint32_t owner = ((y / 8u) * bxn + x / 8u) % n;
            const size_t o = ((size_t)y * p->width + x) * 3u;
            memcpy(host_out + o, sh[owner].img.data() + o, 3u * sizeof(float));
        }
    for (Shard& x : sh) seg += x.seg;
    if (stats) {
        stats->segments = seg;
        stats->samples = (uint64_t)p->width * p->height * p->samples_per_pixel;
        stats->kernel_ms = ms_max;
    }
    cleanup();
    return RT_OK;
}

int rt_set_option(int option, int64_t value) {
    rthost::clear_error();
    if (option < 0 || option >= RT_OPT_COUNT) return rthost::set_error(RT_ERR_INVALID, "unknown option");
    bool ok = true;
    switch (option) {
        case RT_OPT_TUNE:  // only the bits this build honours (the product: exact ones only)
            ok = value >= 0 && value <= 0xffffffffll && ((uint64_t)value & ~(uint64_t)kTuneAccepted) == 0u;
            break;
        case RT_OPT_GROUP: ok = value >= 0 && value <= 64; break;
        case RT_OPT_STACK_LDS: ok = value >= 0 && value <= 96; break;
        case RT_OPT_SAMPLE_BUFFER_MB: ok = value >= 0 && value <= (1ll << 30); break;
        case RT_OPT_HRPP_SLOT_BITS: ok = value >= -1 && value <= 28; break;
        case RT_OPT_LAUNCH_LOG: ok = value == 0 || value == 1; break;
        case RT_OPT_BVH_BUILD: ok = value >= 0 && value <= 2; break;
        case RT_OPT_GUIDE: ok = value >= 0 && value <= 256; break;
        case RT_OPT_BVH_SHAPE: ok = value == 0 || value == 1; break;
    }
    if (!ok) return rthost::set_error(RT_ERR_INVALID, "option value out of range");
    g_opt[option].store(value, std::memory_order_relaxed);
    return RT_OK;
}

int rt_get_option(int option, int64_t* value) {
    rthost::clear_error();
    if (option < 0 || option >= RT_OPT_COUNT || !value) return rthost::set_error(RT_ERR_INVALID, "unknown option");
    *value = opt(option);
    return RT_OK;
}

int rt_scene_trace_time(rt_scene_handle s, double* total_ms, uint64_t* launches, int reset) {
    rthost::clear_error();
    if (!s || !total_ms || !launches) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    DeviceGuard g(s->device);
    std::lock_guard<std::mutex> lock(s->mu);
    double sum = 0.0;
    for (int i = 0; i < s->ev_count; ++i) {
        hipError_t e = hipEventSynchronize(s->ev[i][1]);
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
        float ms = 0.0f;
        if ((e = hipEventElapsedTime(&ms, s->ev[i][0], s->ev[i][1])) != hipSuccess) return hip_fail(e, "hipEventElapsedTime");
        sum += ms;
    }
    *total_ms = sum;
    *launches = (uint64_t)s->ev_count;
    if (s->ev_overflow) {
        if (reset) {
            s->ev_count = 0;
            s->ev_overflow = false;
        }
        return rthost::set_error(RT_ERR_INVALID, "more than 256 launches since the last reset: timing incomplete");
    }
    if (reset) s->ev_count = 0;
    return RT_OK;
}

#ifdef RT_PROFILE_REGIONS
// Profiling build only (not in include/rt.h): render only the 8x8-block rows [r0, r1) of later
// launches (tools/region_profile.py --rows); r1 = ~0u restores the whole frame.
int rt_prof_rows(uint32_t r0, uint32_t r1) {
    g_prof_rows[0] = r0;
    g_prof_rows[1] = r1;
    return RT_OK;
}
#endif

int rt_device_kat(int op, const float* in, float* out, uint32_t n) {
    rthost::clear_error();
    if (!in || !out) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    if (op < 0 || op > 4) return rthost::set_error(RT_ERR_INVALID, "unknown KAT op");
    int rc = check_device(0);
    if (rc) return rc;
    if (n == 0) return RT_OK;
    DeviceGuard g(0);
    const size_t in_floats = (size_t)n * (op <= 1 ? 14u : (op == 2 || op == 4 ? 3u : 12u)),
                 out_floats = (size_t)n * 2u;
    float *din = nullptr, *dout = nullptr;
    hipError_t e = hipMalloc(&din, in_floats * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&dout, out_floats * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(din, in, in_floats * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        (void)hipGetLastError();
        hipLaunchKernelGGL(kat_eval, dim3((n + 63u) / 64u), dim3(64), 0, nullptr, op, din, dout, n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, out_floats * sizeof(float), hipMemcpyDeviceToHost);
    if (din) (void)hipFree(din);
    if (dout) (void)hipFree(dout);
    if (e != hipSuccess) return hip_fail(e, "kat_eval");
    return RT_OK;
}

int rt_device_numeric_eval(int op, const double* a, const double* b, double* out, uint32_t n) {
    rthost::clear_error();
    if (!a || !out) return rthost::set_error(RT_ERR_INVALID, "NULL argument");
    int rc = check_device(0);
    if (rc) return rc;
    if (n == 0) return RT_OK;
    DeviceGuard g(0);
    double *da = nullptr, *db = nullptr, *dout = nullptr;
    size_t bytes = (size_t)n * sizeof(double);
    hipError_t e = hipMalloc(&da, bytes);
    if (e == hipSuccess && b) e = hipMalloc(&db, bytes);
    if (e == hipSuccess) e = hipMalloc(&dout, bytes);
    if (e == hipSuccess) e = hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && b) e = hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        (void)hipGetLastError();
        hipLaunchKernelGGL(numeric_eval, dim3((n + 255u) / 256u), dim3(256), 0, nullptr, op, da, db, dout, n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
    if (da) (void)hipFree(da);
    if (db) (void)hipFree(db);
    if (dout) (void)hipFree(dout);
    if (e != hipSuccess) return hip_fail(e, "numeric_eval");
    return RT_OK;
}

}  // extern "C"
#endif  // RT_INSTANCES_TU
