#!/usr/bin/env bash
# Round 6, call 16: leaf postponement in sphere-only BVHs (C3's sphere cluster; make variant NAME=postsph
# VFLAGS=-DRT_POSTPONE_SPH=1, with lower.cpp's kBvhSphOnly wrapper flag) at q = 8 (default), 4 and 12
# sixteenths (RT_OPT_TUNE bits 24-27), against the product (same lowering); then the sphere-preset
# parity cases on the variant.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s16
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
run ab.log 600 bash tools/ab_session.sh r06_postsph "C3:100 C1" $L/librtamd.so $L/librtamd_postsph.so \
    $L/librtamd_postsph.so:0x04000000 $L/librtamd_postsph.so:0x0c000000
run parity.log 900 env RT_LIBRARY=$L/librtamd_postsph.so python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread -k "golden or other_seeds or every_feature or full_workload or c1_full or bvh_shapes or prebuilt or degenerate"
echo "== done" | tee -a "$OUT/session.log"
