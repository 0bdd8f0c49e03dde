#!/usr/bin/env bash
# Round-2 evidence for the bench line: rocprofv3 kernel trace + stats of the default bench
# command, then PMC passes over one C3 frame (bench.py --steps 1 --warmup 0), each in its
# own run: memory-side traffic (FETCH_SIZE, WRITE_SIZE), and the VALU roofline counters
# tools/valu_roofline.py reads (issue activity, lane cycles, instruction mix, waits).
# Usage: bash tools/profile_r02.sh <tag>
set -u
cd "$(dirname "$0")/.."
TAG="${1:-r02}"
OUT="gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <seconds> <cmd...>
    local name="$1" secs="$2"
    shift 2
    echo "== $name" | tee -a "$OUT/session.log"
    timeout -k 10 -s KILL "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/session.log"
    grep '^{' "$OUT/$name.log" | tail -n 1
    if [ $rc -ne 0 ]; then
        tail -n 20 "$OUT/$name.log"
        echo "== stopping" | tee -a "$OUT/session.log"
        exit $rc
    fi
}
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
step bench_trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o bench --output-format csv -- $B
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o bench --output-format csv -- $B
step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d "$OUT/sq" -o bench --output-format csv -- $B
step pmc_wait 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM \
    SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d "$OUT/wait" -o bench --output-format csv -- $B
step pmc_mix 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQC_ICACHE_HITS SQC_ICACHE_MISSES -d "$OUT/mix" -o bench \
    --output-format csv -- $B
echo "== profile done" | tee -a "$OUT/session.log"
