#!/usr/bin/env bash
# Round-end evidence on the GPU box: the default bench line (C3), a bench line per
# BASELINE config, then tools/profile_bench.sh (rocprofv3 kernel trace + PMC passes).
# Every GPU step has its own time limit; any failure stops the session.
# Usage: bash tools/measure_session.sh <tag> [configs...]
set -u
cd "$(dirname "$0")/.."
TAG="${1:-r01}"
shift || true
CONFIGS="${*:-C1 C2 C4 C5}"
mkdir -p gpurun_out/measure
export TMPDIR=/tmp

step() {  # step <name> <seconds> <cmd...>
    local name="$1" secs="$2"
    shift 2
    echo "== $name" | tee -a gpurun_out/measure/session.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/measure/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/measure/session.log
    grep '^{' "gpurun_out/measure/$name.log" | tail -n 1 > "gpurun_out/measure/$name.json"
    if [ $rc -ne 0 ]; then
        tail -n 20 "gpurun_out/measure/$name.log"
        echo "== stopping" | tee -a gpurun_out/measure/session.log
        exit $rc
    fi
}

step bench_C3 600 python bench.py --steps 3 --warmup 1
for c in $CONFIGS; do
    step "bench_$c" 600 python bench.py --config "$c" --steps 2 --warmup 1
done
timeout -k 10 1000 bash tools/profile_bench.sh "$TAG" || exit $?
echo "== measure done" | tee -a gpurun_out/measure/session.log
