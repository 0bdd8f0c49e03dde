#!/usr/bin/env bash
# Round 6, call 7: the product with the relaxed triangle rule in the replay pass only (C4 against
# the nozd variant of call 6 and against the 3-wave instance, RT_OPT_TUNE kModeW3 = 0x40); the C3
# band profile again, now with each band's blocks as the whole pool (rt_prof_rows offsets the block
# map; call 5 claimed and skipped the other units, which inflated Refill); parity of the C4 cases.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s7
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
run ab_c4.log 600 bash tools/ab_session.sh r06_c4w "C4:50 C4:200" $L/librtamd.so $L/librtamd_nozd.so $L/librtamd.so:0x40
run bands.log 600 env RT_LIBRARY=$L/librtamd_prof.so python3 -u tools/region_profile.py --config C3 --spp 64 --bands 10
run parity.log 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "zero_direction or C4 or c4 or suspending or every_feature or replay or golden"
echo "== done" | tee -a "$OUT/session.log"
