#!/usr/bin/env python3
"""The trace kernel's vector-ALU roofline from rocprofv3 PMC passes (bench.py roofline.valu).

    python3 tools/valu_roofline.py <prof_dir> <config> <segments_per_frame> [--out profiles/pmc_valu.json]

<prof_dir> holds rocprofv3 --pmc runs (subdirectories with *_counter_collection.csv) of
ONE frame of <config>; counters are summed over every trace_samples dispatch. Computed:

  valu_issue  = 4 * SQ_ACTIVE_INST_VALU / simd_cycles, simd_cycles = 1024 SIMDs *
                GRBM_GUI_ACTIVE / 8 (GRBM_GUI_ACTIVE sums the 8 XCDs; ACTIVE_INST_*
                count quad-cycles): the fraction of SIMD cycles the VALU is issuing.
                Calibrated on the box by tools/valu_rate.hip under the same counters
                (profiles/r02/valu_rate_pmc.csv): independent wave64 VALU streams at
                8 waves / SIMD take 4.4-4.9 SIMD cycles per instruction (v_fma_f64,
                v_pk_fma_f32) and read valu_issue = 0.85-0.91, so 1.0 is the ceiling;
  lane_util   = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU): the mean fraction of
                the 64 lanes active in an issued VALU instruction;
  useful_frac = valu_issue * lane_util: the fraction of the VALU's lane throughput
                spent on active lanes — the roofline fraction the kernel reaches.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("config")
    ap.add_argument("segments", type=float, help="ray segments of the profiled frame")
    ap.add_argument("--out", default="profiles/pmc_valu.json")
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    s = sums(a.prof_dir)
    insts = s["SQ_INSTS_VALU"]
    f64_n = s.get("SQ_INSTS_VALU_ADD_F64", 0) + s.get("SQ_INSTS_VALU_MUL_F64", 0) + s.get("SQ_INSTS_VALU_FMA_F64", 0)
    trans = s.get("SQ_INSTS_VALU_TRANS_F32", 0) + s.get("SQ_INSTS_VALU_TRANS_F64", 0)
    simd_cycles = SIMDS * s["GRBM_GUI_ACTIVE"] / 8.0
    lane = s["SQ_THREAD_CYCLES_VALU"] / (64.0 * s["SQ_ACTIVE_INST_VALU"])
    issue = 4.0 * s["SQ_ACTIVE_INST_VALU"] / simd_cycles
    out = {
        "config": a.config,
        "kernel": "trace_samples",
        "bound": "valu",
        "valu_issue": issue,
        "lane_util": lane,
        "useful_frac": issue * lane,
        "valu_inst_per_segment": insts / a.segments,
        "salu_inst_per_segment": s.get("SQ_INSTS_SALU", 0) / a.segments,
        "f64_share": f64_n / insts,
        "trans_share": trans / insts,
        "wait_any": s.get("SQ_WAIT_ANY", 0) / s["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in s else None,
        "wait_inst_any": s.get("SQ_WAIT_INST_ANY", 0) / s["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in s else None,
        "icache_miss_rate": (s["SQC_ICACHE_MISSES"] / (s["SQC_ICACHE_HITS"] + s["SQC_ICACHE_MISSES"])
                             if "SQC_ICACHE_HITS" in s else None),
        "calibration": "profiles/r02/valu_rate_pmc.csv (tools/valu_rate.hip: saturated streams read valu_issue "
                       "0.85-0.91 at 4.4-4.9 SIMD cycles per wave64 instruction)",
        "method": "rocprofv3 --pmc passes over one frame (tools/profile_r02.sh); see tools/valu_roofline.py",
        "source": a.prof_dir + (f" ({a.label})" if a.label else ""),
        "counters": s,
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters"}, indent=1))


if __name__ == "__main__":
    main()
