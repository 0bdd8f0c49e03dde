#!/usr/bin/env bash
# Round 6, call 5: (1) bisect of a C4 slowdown that the reference-shaped tree shows (77.6 vs 68.2 ms
# per 50-spp frame against round 5, r06_sah A/B): the libraries of commits ce98c15, 1a3ff1b, 7a08d8c,
# c636c2e (built from those commits: make all), the current one with bvh_shape=1 and the default;
# (2) C3's mid-frame throughput dip: the region profile in 10 bands of block rows.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s5
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
run ab.log 600 bash tools/ab_session.sh r06_c4bisect "C4:50" $L/librtamd_r05.so $L/librtamd_b_ce98c15.so $L/librtamd_b_1a3ff1b.so \
    $L/librtamd_b_7a08d8c.so $L/librtamd.so:bvh_shape=1 $L/librtamd.so
run bands.log 600 env RT_LIBRARY=$L/librtamd_prof.so python3 -u tools/region_profile.py --config C3 --spp 64 --bands 10
run whole.log 300 env RT_LIBRARY=$L/librtamd_prof.so python3 -u tools/region_profile.py --config C3 --spp 64
echo "== done" | tee -a "$OUT/session.log"
