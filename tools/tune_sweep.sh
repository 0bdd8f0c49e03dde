#!/usr/bin/env bash
# Bench the trace kernel under RT_TUNE / RT_LIBRARY variants (diagnostics).
# Usage: bash tools/tune_sweep.sh <outdir> "<label>:<env assignments>" ...
set -u
cd "$(dirname "$0")/.."
OUT="$1"
shift
mkdir -p "$OUT"
for spec in "$@"; do
    label="${spec%%:*}"
    envs="${spec#*:}"
    env $envs timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/$label.log" 2>&1
    rc=$?
    v=$(grep '^{' "$OUT/$label.log" | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(f"{j[\"value\"]:.1f} Msamples/s kernel {j[\"roofline\"][\"kernel_ms\"]:.1f} ms")' 2>/dev/null)
    echo "$label rc=$rc $v" | tee -a "$OUT/summary.txt"
    [ $rc -eq 0 ] || exit $rc
done
