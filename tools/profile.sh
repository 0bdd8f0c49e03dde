#!/usr/bin/env bash
# Evidence for a bench line (run through gpurun from the repo root):
#   bash tools/profile.sh <tag> [config]
# rocprofv3 kernel trace + stats of the bench command, then PMC passes over one frame of
# the config (bench.py --steps 1 --warmup 0), each in its own run: memory-side traffic
# (FETCH_SIZE, WRITE_SIZE) and the VALU roofline counters tools/valu_roofline.py reads
# (issue quad-cycles incl. dual issue, lane cycles, instruction mix, waits). The md5 of the
# librtamd.so profiled is recorded, so bench.py only quotes these counters for that library.
set -u
cd "$(dirname "$0")/.."
TAG="${1:?tag}"
CFG="${2:-C3}"
OUT="gpurun_out/prof_${TAG}_$CFG"
mkdir -p "$OUT"
export TMPDIR=/tmp
md5sum raytracinginoneweekendinrust_amd/_lib/librtamd.so | cut -d' ' -f1 > "$OUT/library_md5"

step() {  # step <name> <seconds> <cmd...>
    local name="$1" secs="$2"
    shift 2
    echo "== $name $(date +%T)" | tee -a "$OUT/session.log"
    timeout -k 10 -s KILL "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/session.log"
    grep '^{' "$OUT/$name.log" | tail -n 1 | cut -c1-300
    if [ $rc -ne 0 ]; then
        tail -n 20 "$OUT/$name.log"
        echo "== stopping" | tee -a "$OUT/session.log"
        exit $rc
    fi
}
B="python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline"
step bench_trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv \
    -- python3 bench.py --config "$CFG" --no-cpu-baseline
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o bench --output-format csv -- $B
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o bench --output-format csv -- $B
step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE \
    -d "$OUT/sq" -o bench --output-format csv -- $B
step pmc_wait 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM \
    SQ_INSTS_BRANCH SQ_BUSY_CYCLES -d "$OUT/wait" -o bench --output-format csv -- $B
step pmc_mix 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 \
    SQ_INSTS_VALU_MUL_F32 -d "$OUT/mix" -o bench --output-format csv -- $B
echo "== profile done" | tee -a "$OUT/session.log"
