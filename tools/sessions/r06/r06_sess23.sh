#!/usr/bin/env bash
# Round 6, call 23: the stack top read at the start of each BVH trip, beside the node loads, and taken by
# the pop loop's first iteration (make variant NAME=popf VFLAGS=-DRT_POP_PREFETCH=1; the sphere-BVH presets)
# against the product (81d8c5fe), then the sphere-preset parity cases on the variant.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s23
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <log> <seconds> <cmd...>
    local log="$1" secs="$2"
    shift 2
    echo "== $log $(date +%T)" | tee -a "$OUT/session.log"
    timeout -k 10 -s KILL "$secs" "$@" > "$OUT/$log" 2>&1
    local rc=$?
    echo "== $log rc=$rc" | tee -a "$OUT/session.log"
    if [ $rc -ne 0 ]; then
        tail -n 30 "$OUT/$log"
        exit $rc
    fi
}
L=raytracinginoneweekendinrust_amd/_lib
run ab.log 600 bash tools/ab_session.sh r06_popf "C3:100 C3 C1" $L/librtamd.so $L/librtamd_popf.so
run parity.log 900 env RT_LIBRARY=$L/librtamd_popf.so python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kats.py -x -v \
    --timeout 300 --timeout-method thread -k "golden or other_seeds or every_feature or full_workload or c1_full or bvh_shapes or prebuilt or degenerate or depth or kats or zero_direction"
echo "== done" | tee -a "$OUT/session.log"
