#!/usr/bin/env bash
# Round 6, call 3: why the cross-lane traversal lost (C3 100 spp: 91.3 vs 83.2 ms): region profiles
# of the shared and the per-lane loop (make single NAME=prof_share VFLAGS=-DRT_PROFILE_REGIONS,
# NAME=prof_noshare VFLAGS="-DRT_PROFILE_REGIONS -DRT_SHARE=0"), then A/B of three hand-over
# policies (make variant NAME=sh_norefresh VFLAGS=-DRT_SHARE_REFRESH=0, sh_max16 -DRT_SHARE_MAXWORK=16,
# sh_minsp2 -DRT_SHARE_MINSP=2) against the per-lane loop.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s3
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
run regions_share.log 300 env RT_LIBRARY=$L/librtamd_prof_share.so python3 -u tools/region_profile.py --config C3 --spp 64
run regions_noshare.log 300 env RT_LIBRARY=$L/librtamd_prof_noshare.so python3 -u tools/region_profile.py --config C3 --spp 64
run ab.log 600 bash tools/ab_session.sh r06_share2 "C3:100" $L/librtamd_noshare.so $L/librtamd.so $L/librtamd_sh_norefresh.so \
    $L/librtamd_sh_max16.so $L/librtamd_sh_minsp2.so
echo "== done" | tee -a "$OUT/session.log"
