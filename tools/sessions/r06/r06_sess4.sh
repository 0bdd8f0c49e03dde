#!/usr/bin/env bash
# Round 6, call 4: the SAH-rebuilt BVH4 over the reference tree's leaf nodes (RT_OPT_BVH_SHAPE 0, the
# new default) against the reference tree collapsed as built (bvh_shape=1, rounds 1-5) and the round-5
# library (librtamd_r05.so, md5 4dba1833..., rebuilt from commit 576fd0b); then the parity tests.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s4
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
L=raytracinginoneweekendinrust_amd/_lib
run ab.log 900 bash tools/ab_session.sh r06_sah "C3:100 C1 C4:50 C2:32 C5:64" $L/librtamd.so $L/librtamd.so:bvh_shape=1 $L/librtamd_r05.so
run parity.log 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kats.py -x -v --timeout 300 --timeout-method thread \
    -k "golden or other_seeds or traversal_audit or pruned_traversal or every_feature or zero_direction or depth_limits or degenerate or full_workload or c1_full or shapes or stack_spill or suspending or kats or zero_direction_components"
echo "== done" | tee -a "$OUT/session.log"
