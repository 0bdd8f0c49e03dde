#!/usr/bin/env bash
# One GPU-box session: smoke -> GPU parity tests -> bench (+ optional profiling).
# Every GPU step has its own time limit; a fault / abort / timeout (exit >= 124
# or a signal) stops the session, ordinary test failures (exit 1) do not.
# Usage: bash tools/gpu_session.sh [tests|bench|profile|all] [extra pytest args]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
MODE="${1:-all}"
shift || true
export TMPDIR=/tmp

run() {  # run <name> <seconds> <cmd...>
    local name="$1" secs="$2"
    shift 2
    echo "== $name: $*" | tee -a gpurun_out/session.log
    local t0=$(date +%s)
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a gpurun_out/session.log
    tail -n 30 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then
        echo "== stopping after $name (rc=$rc)" | tee -a gpurun_out/session.log
        exit $rc
    fi
    return 0
}

if [ -x tools/valu_rate ] && [ "$MODE" = "all" ]; then
    run valu_rate 120 tools/valu_rate
fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [ "$MODE" = "tests" ] || [ "$MODE" = "all" ]; then
    run gpu_tests 1500 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread "$@"
fi
if [ "$MODE" = "bench" ] || [ "$MODE" = "all" ] || [ "$MODE" = "profile" ]; then
    run bench 900 python bench.py --steps 3 --warmup 1
fi
if [ "$MODE" = "profile" ]; then
    run rocprof_trace 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv \
        -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
fi
echo "== session done" | tee -a gpurun_out/session.log
