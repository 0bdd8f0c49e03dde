#!/usr/bin/env bash
# Round 6, call 12: zero-direction rays in triangle-only BVHs on the fast traversal in the fast kernel
# too (make variant_main NAME=zdfast VFLAGS=-DRT_TRI_ZERO_DIR_FAST=1), now that the triangle preset runs
# its spill-free 3-wave instance: A/B against the product on C4 (50 spp, 200 spp, the full frame,
# which includes the streaming replay's tail), then the C4 parity cases on the variant.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s12
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
run ab.log 600 bash tools/ab_session.sh r06_zdfast "C4:50 C4" $L/librtamd_a15.so $L/librtamd.so $L/librtamd_zdfast.so
run parity.log 900 env RT_LIBRARY=$L/librtamd_zdfast.so python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -k "C4 or zero_direction or every_feature or streaming or replay"
run kats.log 300 env RT_LIBRARY=$L/librtamd_zdfast.so python3 -u -m pytest tests/test_gpu_kats.py -x -v --timeout 120 \
    --timeout-method thread
echo "== done" | tee -a "$OUT/session.log"
