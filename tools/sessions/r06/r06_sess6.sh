#!/usr/bin/env bash
# Round 6, call 6: A/B of the BVH-loop variants (make variant NAME=pushbf VFLAGS=-DRT_PUSH_BF=1,
# sort3 -DRT_SORT3=1, pushbf_sort3 both) and of the ray_route switches behind the C4 slowdown of
# commit 1a3ff1b (nozd -DRT_TRI_ZERO_DIR=0, notnum -DRT_TNUM=0, nozd_notnum both), all from commit
# "A/B switches for the ray_route changes".
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s6
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
run ab_c4.log 600 bash tools/ab_session.sh r06_route "C4:50" $L/librtamd.so $L/librtamd_nozd.so $L/librtamd_notnum.so \
    $L/librtamd_nozd_notnum.so $L/librtamd_sort3.so
run ab_loop.log 600 bash tools/ab_session.sh r06_loop "C3:100 C1" $L/librtamd.so $L/librtamd_pushbf.so $L/librtamd_sort3.so \
    $L/librtamd_pushbf_sort3.so
echo "== done" | tee -a "$OUT/session.log"
