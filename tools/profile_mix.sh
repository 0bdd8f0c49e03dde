#!/usr/bin/env bash
# Where the trace kernel's cycles go (round 2): the region profiler (librtamd_prof.so)
# and PMC passes for the VALU instruction mix, SALU / fetch and the instruction cache,
# each pass its own short run (C3 at reduced spp). Usage: bash tools/profile_mix.sh <tag> [config] [spp]
set -u
cd "$(dirname "$0")/.."
TAG="${1:-mix}"
CFG="${2:-C3}"
SPP="${3:-64}"
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
    tail -n 40 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then
        echo "== stopping" | tee -a "$OUT/session.log"
        exit $rc
    fi
}
R="python3 tools/render_once.py --config $CFG --spp $SPP"
step regions 300 env RT_LIBRARY=raytracinginoneweekendinrust_amd/_lib/librtamd_prof.so python3 tools/region_profile.py --config "$CFG" --spp "$SPP"
step pmc_mix1 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 \
    SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -d "$OUT/mix1" -o run --output-format csv -- $R
step pmc_mix2 120 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_INSTS_SALU \
    SQ_INST_CYCLES_SALU SQ_IFETCH SQ_ACTIVE_INST_VALU -d "$OUT/mix2" -o run --output-format csv -- $R
step pmc_wait 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU \
    SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAIT_INST_LDS -d "$OUT/wait" -o run --output-format csv -- $R
step pmc_icache 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d "$OUT/icache" -o run --output-format csv -- $R
step pmc_grbm 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM \
    -d "$OUT/grbm" -o run --output-format csv -- $R
echo "== profile done" | tee -a "$OUT/session.log"
