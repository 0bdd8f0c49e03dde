#!/usr/bin/env bash
# Round 6, call 21: the sphere-BVH presets without the clamp of a visited child's key (make variant
# NAME=noclamp VFLAGS=-DRT_NO_KEY_CLAMP=1: ray_route's magnitude rule, P in the wrapper's rank[0]) against the
# product (81d8c5fe; the variant links the lowering that stores P), then the sphere-preset parity cases on the variant; then a whole-frame region
# profile of C3 at 64 spp (make prof: the product's device code with the region counters).
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s21
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
run ab.log 600 bash tools/ab_session.sh r06_noclamp "C3:100 C3 C1" $L/librtamd.so $L/librtamd_noclamp.so
run parity.log 900 env RT_LIBRARY=$L/librtamd_noclamp.so python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kats.py -x -v \
    --timeout 300 --timeout-method thread -k "golden or other_seeds or every_feature or full_workload or c1_full or bvh_shapes or prebuilt or degenerate or depth or kats or zero_direction"
run regions_c3.log 600 env RT_LIBRARY=$L/librtamd_prof.so python3 -u tools/region_profile.py --config C3 --spp 64
echo "== done" | tee -a "$OUT/session.log"
