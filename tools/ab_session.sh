#!/usr/bin/env bash
# Same-box A/B of librtamd builds over several configs (run through gpurun from the repo root):
#   bash tools/ab_session.sh <tag> "<C3:100 C1 C2:64 ...>" lib1.so lib2.so ...
# Each config (name[:spp]) runs tools/ab_time.py twice, the libraries in the given order and then
# reversed, so a clock drift during the session shows up instead of favouring one build. Every
# run has its own time limit; the session stops at the first failure. Logs: gpurun_out/ab_<tag>/.
set -u
cd "$(dirname "$0")/.."
TAG="${1:?tag}"
CFGS="${2:?configs}"
shift 2
OUT="gpurun_out/ab_$TAG"
mkdir -p "$OUT"
rev=()
for ((i = $#; i >= 1; i--)); do rev+=("${!i}"); done
for c in $CFGS; do
    name="${c%%:*}"
    spp=""
    [ "$name" != "$c" ] && spp="--spp ${c#*:}"
    for pass in fwd rev; do
        if [ $pass = fwd ]; then libs=("$@"); else libs=("${rev[@]}"); fi
        echo "== $c $pass $(date +%T)" | tee -a "$OUT/session.log"
        timeout -k 10 300 python3 -u tools/ab_time.py --config "$name" $spp --reps 5 "${libs[@]}" \
            >> "$OUT/ab_$name.log" 2>&1
        rc=$?
        tail -n ${#libs[@]} "$OUT/ab_$name.log" | tee -a "$OUT/session.log"
        if [ $rc -ne 0 ]; then
            echo "== rc=$rc, stopping" | tee -a "$OUT/session.log"
            tail -n 20 "$OUT/ab_$name.log"
            exit $rc
        fi
    done
done
echo "== ab done" | tee -a "$OUT/session.log"
