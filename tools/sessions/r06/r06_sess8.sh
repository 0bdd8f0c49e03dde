#!/usr/bin/env bash
# Round 6, call 8: non-temporal sample-buffer stores (make variant NAME=sbufnt VFLAGS=-DRT_SBUF_NT=1)
# against the product on C3 and C4, the 3-wave instances (RT_OPT_TUNE kModeW3 = 0x40) beside them,
# and each variant's HBM bytes per frame (FETCH_SIZE / WRITE_SIZE in separate passes over
# tools/ab_time.py --reps 1, read by tools/pmc_ab.py).
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s8
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
run ab.log 600 bash tools/ab_session.sh r06_sbufnt "C3:100 C4:50" $L/librtamd.so $L/librtamd_sbufnt.so $L/librtamd.so:0x40
pmc() {  # pmc <name> <config:spp> <lib spec>
    local name="$1" cfg="${2%%:*}" spp="${2##*:}" spec="$3"
    run "pmc_${name}_fetch.log" 180 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc/$name/fetch" -o run --output-format csv \
        -- python3 tools/ab_time.py --config "$cfg" --spp "$spp" --reps 1 "$spec"
    run "pmc_${name}_write.log" 180 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc/$name/write" -o run --output-format csv \
        -- python3 tools/ab_time.py --config "$cfg" --spp "$spp" --reps 1 "$spec"
}
pmc c3_product C3:100 $L/librtamd.so
pmc c3_sbufnt C3:100 $L/librtamd_sbufnt.so
pmc c3_3waves C3:100 $L/librtamd.so:0x40
pmc c4_product C4:50 $L/librtamd.so
pmc c4_sbufnt C4:50 $L/librtamd_sbufnt.so
pmc c4_3waves C4:50 $L/librtamd.so:0x40
python3 tools/pmc_ab.py "$OUT"/pmc/* | tee "$OUT/traffic.txt"
echo "== done" | tee -a "$OUT/session.log"
