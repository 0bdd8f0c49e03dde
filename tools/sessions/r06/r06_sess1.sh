#!/usr/bin/env bash
# Round 6 (run after call 9, on the library of commit a15b17a, md5 a50038f8...): the new multi-process cases (8 ranks on one GPU: the bench over ipc and shm,
# the position-coded gather at world 8), then the whole GPU suite (with the round-6 zero-direction
# cases on the triangle BVH), then the C3 and C4 bench lines.
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s1
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
run multiproc.log 900 python3 -u -m pytest tests/test_gpu_multiprocess.py -v --timeout 500 --timeout-method thread
run gpu_tests.log 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    --ignore tests/test_gpu_multiprocess.py
run bench_C3.log 300 python3 -u bench.py --config C3
run bench_C4.log 300 python3 -u bench.py --config C4
echo "== done" | tee -a "$OUT/session.log"
