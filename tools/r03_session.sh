#!/usr/bin/env bash
# Round-3 GPU sessions (run through gpurun from the repo root): bash tools/r03_session.sh <name> [args]
# Every GPU step runs under its own time limit; the script stops at the first failure.
set -u
cd "$(dirname "$0")/.."
NAME="${1:?session name}"
shift
OUT="gpurun_out/r03_$NAME"
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <log name> <seconds> <cmd...>
    local name="$1" secs="$2"
    shift 2
    echo "== $name $(date +%T)" | tee -a "$OUT/session.log"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)" | tee -a "$OUT/session.log"
    grep '^{' "$OUT/$name.log" | tail -n 3 | cut -c1-400
    if [ $rc -ne 0 ]; then
        tail -n 30 "$OUT/$name.log"
        echo "== stopping" | tee -a "$OUT/session.log"
        exit $rc
    fi
}
pmc() {  # pmc <log name> <counters...> -- <cmd...>
    local name="$1"
    shift
    local ctr=()
    while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
    shift
    step "pmc_$name" 300 rocprofv3 --pmc "${ctr[@]}" -d "$OUT/pmc_$name" -o run --output-format csv -- "$@"
}
gpu_tests() {
    step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
}
smoke() {
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
}

case "$NAME" in
calib)  # the VALU issue peak, wall clock and PMC
    step valu_rate 600 tools/valu_rate
    for w in 4 8; do
        pmc "fma_w$w" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES \
            SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- tools/valu_rate v_fma_f32 $w 60
    done
    pmc "fma64_w4" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- tools/valu_rate v_fma_f64 4 60
    pmc "pkfma_w4" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- tools/valu_rate v_pk_fma_f32 4 60
    ;;
first)  # round start: GPU suite, smoke, bench, calibration, C3 dual-issue counters
    gpu_tests
    smoke
    step bench 600 python -u bench.py
    step valu_rate 600 tools/valu_rate
    for w in 4 8; do
        pmc "fma_w$w" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES \
            SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- tools/valu_rate v_fma_f32 $w 60
    done
    pmc "pkfma_w4" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- tools/valu_rate v_pk_fma_f32 4 60
    pmc "c3_valu2" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
    ;;
probe)  # dual-issue rules, the C3 region profile and instruction classes of the current kernel
    step valu_rate_w4 600 tools/valu_rate all 4
    step valu_rate_w2 600 tools/valu_rate all 2
    for c in v_max_f32 v_cndmask_b32_e32 v_and_b32 v_mov_b32 v_cmp_lt_f32_e32; do
        pmc "$c" SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE \
            -- tools/valu_rate $c 4 30
    done
    step regions_c3 600 env RT_LIBRARY=raytracinginoneweekendinrust_amd/_lib/librtamd_prof.so \
        python3 tools/region_profile.py --config C3 --spp 64
    B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
    pmc c3_mix1 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 \
        SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_VALU -- $B
    pmc c3_mix2 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 \
        SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU -- $B
    ;;
ab)  # A/B of library builds: bash tools/r03_session.sh ab <config> <spp> lib1.so lib2.so ...
    CFG="$1"; SPP="$2"; shift 2
    step "ab_$CFG" 900 python -u tools/ab_time.py --config "$CFG" --spp "$SPP" --reps 3 "$@"
    ;;
*)
    echo "unknown session $NAME"; exit 2 ;;
esac
echo "== session $NAME done" | tee -a "$OUT/session.log"
