#!/usr/bin/env bash
# Round 6, call 9: sphere and cube leaves read from the BVH leaf node's own line (RT_LEAF_EMBED,
# librtamd_embed.so), the wrapper's root-box test peeled out of the traversal loop onto scalar
# loads (RT_PEEL_WRAPPER, librtamd_peel.so), both (librtamd_embed_peel.so), against the product on
# the sphere-BVH presets; the parity tests of those presets on the combined build.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s9
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
run ab.log 600 bash tools/ab_session.sh r06_embed "C3:100 C1" $L/librtamd.so $L/librtamd_embed.so $L/librtamd_peel.so \
    $L/librtamd_embed_peel.so
run parity.log 900 env RT_LIBRARY=$L/librtamd_embed_peel.so python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -k "golden or other_seeds or every_feature or full_workload or c1_full or bvh_shapes or prebuilt or degenerate"
echo "== done" | tee -a "$OUT/session.log"
