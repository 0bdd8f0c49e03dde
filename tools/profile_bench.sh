#!/usr/bin/env bash
# rocprofv3 evidence for the bench line: kernel trace + stats of the bench command,
# then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) — never combined with
# sys/runtime trace domains. Usage: bash tools/profile_bench.sh <tag> [bench args...]
set -u
cd "$(dirname "$0")/.."
TAG="${1:-r01}"
shift || true
ARGS="${*:---steps 3 --warmup 1}"
OUT="gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <seconds> <cmd...>
    local name="$1" secs="$2"
    shift 2
    echo "== $name" | tee -a "$OUT/session.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/session.log"
    grep '^{' "$OUT/$name.log" | tail -n 1
    if [ $rc -ne 0 ]; then
        tail -n 20 "$OUT/$name.log"
        echo "== stopping" | tee -a "$OUT/session.log"
        exit $rc
    fi
}

step bench_trace 900 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv \
    -- python3 bench.py $ARGS --no-cpu-baseline
step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o bench --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step pmc_write 900 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o bench --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step pmc_sq 900 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d "$OUT/sq" -o bench --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step pmc_wait 900 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM \
    SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d "$OUT/wait" -o bench --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
echo "== profile done" | tee -a "$OUT/session.log"
