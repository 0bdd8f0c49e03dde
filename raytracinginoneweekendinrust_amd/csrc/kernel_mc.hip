// The 4-wave trace_samples instances of the BVH-only preset (C1, C3) and the
// sphere-run preset (C2), compiled from kernel.hip with the memory-clause
// scheduling strategy (Makefile). kernel.hip's
// fast_instance launches them through rt_mc_trace_instance; every other kernel
// and the C ABI live there.
#define RT_INSTANCES_TU 1
#include "kernel.hip"
