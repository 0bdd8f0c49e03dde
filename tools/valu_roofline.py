#!/usr/bin/env python3
"""The trace kernel's vector-ALU roofline and memory traffic from tools/profile.sh's PMC passes.

    python3 tools/valu_roofline.py <prof_dir> [--out-dir profiles/r03] [--calib <valu_rate.log>]

<prof_dir> is one `bash tools/profile.sh <tag> <config>` output (gpurun_out/prof_<tag>_<cfg>): PMC runs
of ONE frame (subdirectories with *_counter_collection.csv; every trace_samples dispatch summed),
the bench JSON line of those runs (config, segments) and the md5 of the librtamd.so profiled.
Writes <out-dir>/pmc_valu_<cfg>.json and pmc_traffic_<cfg>.json, which bench.py quotes only
while that very library is loaded.

The VALU model (measured by tools/valu_rate.hip, DESIGN.md §3 "Roofline"): a gfx950 SIMD issues
VALU work in quad-cycles (4 shader cycles). In one quad-cycle it issues one wave64 VALU
instruction, or two from different waves when both are dual-issuable (plain f32 add / mul / fma,
...: a saturated v_fma_f32 stream runs at 2.2-2.5 cycles per instruction per SIMD with 2+ waves,
reads SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU = 0.43 and issue_quads = 0.94); v_cndmask_e64,
v_max3, packed f32, f64 take the whole quad-cycle (4.1-4.4 cycles), transcendentals two (8.1).
Counters (SQ_ACTIVE_INST_* count quad-cycles; GRBM_GUI_ACTIVE sums the 8 XCDs):

  issue_quads  = (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / (1024 SIMDs x cycles / 4):
                 the fraction of the SIMDs' VALU issue quad-cycles in use (saturated stream: 0.94);
  dual_issue   = SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU;
  lane_util    = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU): active lanes per issued instruction
                 (the calibration stream reads exactly 1.0);
  useful_frac  = SQ_THREAD_CYCLES_VALU / (1024 x cycles x 32): useful lane-operations against the
                 measured f32 peak of 32 lanes per cycle per SIMD (a wave64 instruction per 2 cycles)
                 — the roofline fraction the kernel reaches on its actual bound;
  useful_frac_single_issue: the same against 16 lanes per cycle (one instruction per quad-cycle).
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


def bench_line(prof_dir):
    for name in ("pmc_sq.log", "pmc_fetch.log", "bench_trace.log"):
        try:
            for ln in open(os.path.join(prof_dir, name)):
                if ln.startswith("{"):
                    return json.loads(ln)
        except FileNotFoundError:
            continue
    raise SystemExit(f"no bench JSON line in {prof_dir}")


def trace_kernel_ms(prof_dir):
    """Average duration of the fast kernel (trace_samples<0, ...>) in the rocprofv3 --stats summary
    (the streaming replay pass, trace_samples<3, ...>, spans the fast kernel's wall time on its own
    stream and is not the dominant kernel, whatever its total)."""
    for path in glob.glob(os.path.join(prof_dir, "trace", "*kernel_stats.csv")):
        best = None
        for r in csv.DictReader(open(path)):
            if "trace_samples<0," in r["Name"] and (best is None or float(r["TotalDurationNs"]) > float(best["TotalDurationNs"])):
                best = r
        if best:
            return float(best["AverageNs"]) / 1e6, best["Name"]
    return None, None


def calibration(path):
    out = {}
    if path and os.path.exists(path):
        for ln in open(path):
            if ln.startswith("{"):
                j = json.loads(ln)
                out.setdefault(j["op"], {})[str(j["waves_per_simd"])] = j["cycles_per_wave64_inst_per_simd"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--out-dir", default="profiles/r03")
    ap.add_argument("--calib", default="profiles/r03/calib/valu_rate.log")
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    s = sums(a.prof_dir)
    line = bench_line(a.prof_dir)
    cfg = line["config"]["workload"].split()[0]
    segments = line["segments"]
    md5 = open(os.path.join(a.prof_dir, "library_md5")).read().strip()
    cycles = s["GRBM_GUI_ACTIVE"] / 8.0
    insts = s["SQ_INSTS_VALU"]
    quads = SIMDS * cycles / 4.0
    f64_n = s.get("SQ_INSTS_VALU_ADD_F64", 0) + s.get("SQ_INSTS_VALU_MUL_F64", 0) + s.get("SQ_INSTS_VALU_FMA_F64", 0)
    trans = s.get("SQ_INSTS_VALU_TRANS_F32", 0) + s.get("SQ_INSTS_VALU_TRANS_F64", 0)
    kernel_ms, kernel_name = trace_kernel_ms(a.prof_dir)
    valu = {
        "config": cfg,
        "library_md5": md5,
        "kernel": "trace_samples",
        "bound": "valu",
        "issue_quads": (s["SQ_ACTIVE_INST_VALU"] - s.get("SQ_ACTIVE_INST_VALU2", 0.0)) / quads,
        "issue_quads_ceiling": 0.94,
        "dual_issue": s.get("SQ_ACTIVE_INST_VALU2", 0.0) / insts,
        "lane_util": s["SQ_THREAD_CYCLES_VALU"] / (64.0 * insts),
        "useful_frac": s["SQ_THREAD_CYCLES_VALU"] / (SIMDS * cycles * 32.0),
        "useful_frac_single_issue": s["SQ_THREAD_CYCLES_VALU"] / (SIMDS * cycles * 16.0),
        "valu_inst_per_segment": insts / segments,
        "salu_inst_per_segment": s.get("SQ_INSTS_SALU", 0) / segments,
        "f64_share": f64_n / insts if "SQ_INSTS_VALU_ADD_F64" in s else None,
        "trans_share": trans / insts if "SQ_INSTS_VALU_TRANS_F32" in s else None,
        "int32_share": s["SQ_INSTS_VALU_INT32"] / insts if "SQ_INSTS_VALU_INT32" in s else None,
        "wait_any": s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"] if "SQ_WAIT_ANY" in s else None,
        "wait_inst_any": s["SQ_WAIT_INST_ANY"] / s["SQ_WAVE_CYCLES"] if "SQ_WAIT_INST_ANY" in s else None,
        "waves_per_simd": s["SQ_WAVE_CYCLES"] * 4.0 / (SIMDS * cycles) if "SQ_WAVE_CYCLES" in s else None,
        "segments": segments,
        "trace_kernel_ms": kernel_ms,
        "trace_kernel": kernel_name,
        "calibration_cycles_per_wave64_inst": calibration(a.calib),
        "method": "rocprofv3 --pmc passes over one frame (tools/profile.sh), model in tools/valu_roofline.py",
        "source": a.prof_dir + (f" ({a.label})" if a.label else ""),
        "counters": s,
    }
    traffic = {
        "config": cfg,
        "library_md5": md5,
        "kernel": "trace_samples",
        "hbm_bytes_per_launch": (2.0 * s["FETCH_SIZE"] + s["WRITE_SIZE"]) * 1024.0 / max(line["roofline"]["launches_per_step"], 1.0),
        "fetch_bytes": 2.0 * s["FETCH_SIZE"] * 1024.0,
        "write_bytes": s["WRITE_SIZE"] * 1024.0,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes over one frame (bench.py --steps 1 "
                  "--warmup 0); KiB; FETCH_SIZE x2 per the gfx950 note in MI355X_MICROARCH.md",
        "source": a.prof_dir,
    }
    os.makedirs(a.out_dir, exist_ok=True)
    json.dump(valu, open(os.path.join(a.out_dir, f"pmc_valu_{cfg}.json"), "w"), indent=1)
    json.dump(traffic, open(os.path.join(a.out_dir, f"pmc_traffic_{cfg}.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in valu.items() if k not in ("counters", "calibration_cycles_per_wave64_inst")},
                     indent=1))
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
