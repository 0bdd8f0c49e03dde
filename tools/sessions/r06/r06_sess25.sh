#!/usr/bin/env bash
# Round 6, call 25: the whole GPU suite (multi-process tests included) and smoke() on the round's last commit
# (product library 81d8c5fe; the audit library rebuilt with the round's last A/B switches, all off).
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s25
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 &&
    timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "rc=$?" > "$OUT/rc.txt"
md5sum raytracinginoneweekendinrust_amd/_lib/*.so > "$OUT/library_md5"
