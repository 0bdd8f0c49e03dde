// The 4-wave trace_samples instances of the BVH-only preset (C1, C3) and the
// sphere-run preset (C2), compiled from kernel.hip with the memory-clause
// scheduling strategy (Makefile) and philox_block inlined (RT_PHILOX_INLINE: C3
// 109.5 -> 107.7 ms per 100-spp frame, C2 -0.6%, C1 unchanged; the triangle preset
// in kernel.hip keeps the call, inlined it is 8% slower). kernel.hip's
// fast_instance launches them through rt_mc_trace_instance; every other kernel
// and the C ABI live there.
#define RT_INSTANCES_TU 1
#define RT_PHILOX_INLINE 1
#include "kernel.hip"
