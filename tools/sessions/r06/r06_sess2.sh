#!/usr/bin/env bash
# Round 6, call 2: the cross-lane BVH traversal (bvh_run_shared, RT_SHARE=1, the product build of
# commit "Cross-lane BVH traversal") — parity tests of the sphere-BVH presets, then a same-box A/B
# against the per-lane loop (librtamd_noshare.so: make variant NAME=noshare VFLAGS=-DRT_SHARE=0); the same
# for the triangle preset (librtamd_sharetri.so: make variant NAME=sharetri VFLAGS=-DRT_SHARE_TRI=1).
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s2
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <log> <seconds> <cmd...>
    local log="$1" secs="$2"
    shift 2
    echo "== $log $(date +%T)" | tee -a "$OUT/session.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$log" 2>&1
    local rc=$?
    echo "== $log rc=$rc" | tee -a "$OUT/session.log"
    if [ $rc -ne 0 ]; then
        tail -n 30 "$OUT/$log"
        exit $rc
    fi
}
run ab.log 600 bash tools/ab_session.sh r06_share "C3:100 C1" raytracinginoneweekendinrust_amd/_lib/librtamd.so \
    raytracinginoneweekendinrust_amd/_lib/librtamd_noshare.so
run ab_c4.log 600 bash tools/ab_session.sh r06_sharetri "C4:50" raytracinginoneweekendinrust_amd/_lib/librtamd.so \
    raytracinginoneweekendinrust_amd/_lib/librtamd_sharetri.so
run parity.log 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "golden or other_seeds or traversal_audit or pruned_traversal or every_feature or zero_direction or depth_limits or degenerate or full_workload or c1_full"
run parity_sharetri.log 600 env RT_LIBRARY=raytracinginoneweekendinrust_amd/_lib/librtamd_sharetri.so python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "c4 or C4 or zero_direction or suspending or every_feature"
echo "== done" | tee -a "$OUT/session.log"
