#!/usr/bin/env bash
# Round 6, call 17: a triangle-only BVH entered with a NaN closest_so_far scanned in DFS order in the replay
# pass (kernel.hip bvh_hit_nan_tmax) instead of the literal recursion: the parity cases (NaN-closest rays that
# miss and that hit the mesh, zero-direction, replay passes, C4 full-size subsample), then the C4 frame time
# against the previous final library (librtamd_1e22.so = md5 1e223779...) and C3 beside it, the hand-over
# counts, and the kernel trace of a C4 bench run (does the replay pass still end after the fast kernel?).
set -u
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r06_s17
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
run parity.log 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "nan_closest or zero_direction or replay or streaming or full_workload or suspending or every_feature"
run ab.log 600 bash tools/ab_session.sh r06_nanscan "C4 C3:100" $L/librtamd_1e22.so $L/librtamd.so
run replay_count.log 300 python3 -u tools/replay_count.py C4
run trace.log 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv \
    -- python3 bench.py --config C4 --no-cpu-baseline
echo "== done" | tee -a "$OUT/session.log"
