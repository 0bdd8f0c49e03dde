#!/usr/bin/env bash
# A/B session on the GPU box: GPU parity tests, then render_once timings of one
# config under several environments (RT_LAUNCH_LOG=1 prints the launched instance
# and its occupancy). A fault / abort / timeout stops it.
# Usage: bash tools/ab_session.sh [tests|notests] CONFIG SPP VARIANT...
#   VARIANT: comma-separated env assignments, e.g. RT_TUNE=16 or
#            RT_LIBRARY=raytracinginoneweekendinrust_amd/_lib/librtamd_w3.so,RT_TUNE=0
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS="$1"; CFG="$2"; SPP="$3"
shift 3

run() {  # run <name> <seconds> <cmd...>
    local name="$1" secs="$2"
    shift 2
    echo "== $name: $*" | tee -a gpurun_out/ab_session.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/ab_session.log
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then
        echo "== stopping after $name (rc=$rc)" | tee -a gpurun_out/ab_session.log
        exit $rc
    fi
    return 0
}

if [ "$TESTS" = "tests" ]; then
    run gpu_tests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
fi
i=0
for T in "$@"; do
    i=$((i + 1))
    run "ab_${CFG}_${i}" 300 env ${T//,/ } RT_LAUNCH_LOG=1 python tools/render_once.py --config "$CFG" --spp "$SPP" --reps 2
done
echo "== ab done" | tee -a gpurun_out/ab_session.log
