#!/usr/bin/env python3
"""The trace kernel's vector-ALU roofline from rocprofv3 PMC passes (bench.py roofline.valu).

    python3 tools/valu_roofline.py <prof_dir> <config> <segments_per_frame> [--spp-scale S] [--out profiles/pmc_valu.json]

<prof_dir> holds rocprofv3 --pmc runs (subdirectories with *_counter_collection.csv) of
ONE frame of <config>; counters are summed over every trace_samples dispatch. Computed:

  lane_util   = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU): the mean fraction of
                the 64 lanes active in an issued VALU instruction;
  simd_cycles = 1024 SIMDs * GRBM_GUI_ACTIVE / 8 (GRBM_GUI_ACTIVE sums the 8 XCDs);
  valu_active = 4 * SQ_ACTIVE_INST_VALU / simd_cycles (ACTIVE_INST_* count quad-cycles):
                the hardware's VALU-issue-active fraction;
  valu_pipe   = sum over instruction classes of count * cycles per wave64 instruction at
                saturation (profiles/r02/valu_rate.jsonl, tools/valu_rate.hip: measured on
                the box) / simd_cycles: the fraction of VALU throughput the mix consumes;
  useful      = valu_pipe * lane_util: the fraction of the VALU's lane throughput doing
                the work of active lanes (the roofline fraction the kernel actually reaches).
"""
import argparse
import collections
import csv
import glob
import json
import os

SIMDS = 1024


def sums(prof_dir):
    agg = collections.defaultdict(float)
    for path in glob.glob(os.path.join(prof_dir, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            if "trace_samples" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    return dict(agg)


def calibration(path):
    """cycles per wave64 instruction of each class at saturation (8 waves / SIMD)."""
    cyc = {}
    for ln in open(path):
        j = json.loads(ln)
        if j.get("waves_per_simd") == 1 and "op" in j:  # one wave alone already saturates (valu_rate.hip)
            cyc[j["op"]] = j["cycles_per_inst_one_wave"]
    return cyc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("config")
    ap.add_argument("segments", type=float, help="ray segments of the profiled frame")
    ap.add_argument("--calib", default="profiles/r02/valu_rate.jsonl")
    ap.add_argument("--out", default="profiles/pmc_valu.json")
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    s = sums(a.prof_dir)
    cyc = calibration(a.calib)
    f32 = cyc.get("v_fma_f32", 2.7)
    f64 = cyc.get("v_fma_f64", 5.5)
    insts = s["SQ_INSTS_VALU"]
    f64_n = s.get("SQ_INSTS_VALU_ADD_F64", 0) + s.get("SQ_INSTS_VALU_MUL_F64", 0) + s.get("SQ_INSTS_VALU_FMA_F64", 0)
    trans = s.get("SQ_INSTS_VALU_TRANS_F32", 0) + s.get("SQ_INSTS_VALU_TRANS_F64", 0)
    # transcendental and f64 ops: the f64 FMA rate (half the f32 rate); everything else: the f32 rate
    pipe_cycles = (insts - f64_n - trans) * f32 + (f64_n + trans) * f64
    simd_cycles = SIMDS * s["GRBM_GUI_ACTIVE"] / 8.0
    lane = s["SQ_THREAD_CYCLES_VALU"] / (64.0 * s["SQ_ACTIVE_INST_VALU"])
    out = {
        "config": a.config,
        "kernel": "trace_samples",
        "bound": "valu",
        "lane_util": lane,
        "valu_active": 4.0 * s["SQ_ACTIVE_INST_VALU"] / simd_cycles,
        "valu_pipe": pipe_cycles / simd_cycles,
        "useful_frac": pipe_cycles / simd_cycles * lane,
        "valu_inst_per_segment": insts / a.segments,
        "salu_inst_per_segment": s.get("SQ_INSTS_SALU", 0) / a.segments,
        "f64_share": f64_n / insts,
        "trans_share": trans / insts,
        "cycles_per_valu_inst_f32": f32,
        "cycles_per_valu_inst_f64": f64,
        "wait_any": s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in s else None,
        "wait_inst_any": s.get("SQ_WAIT_INST_ANY", 0) / s["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in s else None,
        "icache_miss_rate": (s["SQC_ICACHE_MISSES"] / (s["SQC_ICACHE_HITS"] + s["SQC_ICACHE_MISSES"])
                             if "SQC_ICACHE_HITS" in s else None),
        "method": "rocprofv3 --pmc passes over one frame (tools/profile_mix.sh); cycles per instruction class "
                  "from tools/valu_rate.hip on the same pool; see tools/valu_roofline.py",
        "source": a.prof_dir + (f" ({a.label})" if a.label else ""),
        "counters": s,
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters"}, indent=1))


if __name__ == "__main__":
    main()
