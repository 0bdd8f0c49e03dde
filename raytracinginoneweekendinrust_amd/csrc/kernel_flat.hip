// The trace_samples instances of the flat-list preset (no BVH, no long sphere runs:
// C5), compiled from kernel.hip reading the camera from its
// device copy at each new sample (RT_CAMMEM: 21 fewer words held in SGPRs, C5 +1.8%).
// kernel.hip's fast_instance launches them through rt_flat_trace_instance.
#define RT_INSTANCES_TU 2
#define RT_CAMMEM 1
#include "kernel.hip"
