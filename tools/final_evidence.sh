#!/usr/bin/env bash
# The evidence set for one library build, in one GPU session (run through gpurun from the repo root):
#   bash tools/final_evidence.sh
# 1. tools/profile.sh per config (rocprofv3 kernel trace + the PMC passes), 2. the PMC summaries
# (tools/valu_roofline.py, written where bench.py reads them and copied under gpurun_out/), 3. one
# bench line per config plus a driver-style C3 line, 4. the GPU suite and smoke(). Every GPU step
# has its own time limit; the script stops at the first failure. gpurun allows 20 minutes per call,
# so the session runs in two calls: `bash tools/final_evidence.sh profiles` (1-2), then
# `bash tools/final_evidence.sh bench` (3-4); no argument runs both. ROUND (default r05) names the
# profiles/<ROUND> directory the summaries go to.
set -u
PHASE="${1:-all}"
ROUND="${ROUND:-r05}"
CFGS="${CFGS:-C3 C1 C2 C4 C5}"  # the configs of this call (a call is limited to ~20 minutes)
cd "$(dirname "$0")/.."
OUT=gpurun_out/final_$ROUND
mkdir -p "$OUT/pmc"
export TMPDIR=/tmp
run() {  # run <log> <seconds> <cmd...>
    local log="$1" secs="$2"
    shift 2
    echo "== $log $(date +%T)" | tee -a "$OUT/session.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$log" 2>&1
    local rc=$?
    echo "== $log rc=$rc" | tee -a "$OUT/session.log"
    if [ $rc -ne 0 ]; then
        tail -n 20 "$OUT/$log"
        exit $rc
    fi
}
if [ "$PHASE" != bench ]; then
    for c in $CFGS; do
        run "profile_$c.log" 900 bash tools/profile.sh "final_$ROUND" "$c"
        run "roofline_$c.log" 120 python3 tools/valu_roofline.py "gpurun_out/prof_final_${ROUND}_$c" --out-dir "profiles/$ROUND"
        cp "profiles/$ROUND/pmc_valu_$c.json" "profiles/$ROUND/pmc_traffic_$c.json" "$OUT/pmc/"
    done
fi
if [ "$PHASE" != profiles ]; then
    for c in $CFGS; do
        run "bench_$c.log" 300 python3 -u bench.py --config "$c"
    done
    run bench_driver_style.log 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
    run gpu_tests.log 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
    run smoke.log 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
fi
echo "== final evidence done" | tee -a "$OUT/session.log"
