#!/usr/bin/env bash
# Profiling passes on the GPU box (run after tools/gpu_session.sh has built confidence).
# Kernel trace + stats, then separate --pmc passes (no sys/runtime trace domains).
# Usage: bash tools/profile_session.sh <tag> [config] [spp]
set -u
cd "$(dirname "$0")/.."
TAG="${1:-r01}"
CFG="${2:-C3}"
SPP="${3:-100}"
OUT="gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <seconds> <fatal:0|1> <cmd...>
    local name="$1" secs="$2" fatal="$3"
    shift 3
    echo "== $name" | tee -a "$OUT/session.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/session.log"
    tail -n 12 "$OUT/$name.log"
    if [ $rc -ge 124 ] || { [ "$fatal" = 1 ] && [ $rc -ne 0 ]; }; then
        echo "== stopping" | tee -a "$OUT/session.log"
        exit $rc
    fi
}

step trace 600 1 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 tools/render_once.py --config "$CFG" --spp "$SPP" --reps 2
step list 120 0 rocprofv3 -L
step pmc_fetch 600 0 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
    -- python3 tools/render_once.py --config "$CFG" --spp "$SPP"
step pmc_write 600 0 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
    -- python3 tools/render_once.py --config "$CFG" --spp "$SPP"
step pmc_sq1 600 0 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d "$OUT/sq1" -o run --output-format csv \
    -- python3 tools/render_once.py --config "$CFG" --spp "$SPP"
step pmc_sq2 600 0 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM \
    SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d "$OUT/sq2" -o run --output-format csv \
    -- python3 tools/render_once.py --config "$CFG" --spp "$SPP"
step pmc_tcc 600 0 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
    -d "$OUT/tcc" -o run --output-format csv -- python3 tools/render_once.py --config "$CFG" --spp "$SPP"
echo "== profile done" | tee -a "$OUT/session.log"
