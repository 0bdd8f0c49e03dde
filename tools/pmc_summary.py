#!/usr/bin/env python3
"""Summarise a tools/profile_bench.sh run into profiles/ (kernel stats + PMC sums +
the HBM traffic figure bench.py reports as roofline.traffic).

    python3 tools/pmc_summary.py gpurun_out/prof_r01 profiles/r01 <label>

FETCH_SIZE / WRITE_SIZE are KiB per dispatch; FETCH_SIZE is doubled on gfx950
(MI355X_MICROARCH.md, HBM / rocprofv3 section; checked here on resolve_samples,
whose fetch must equal its 12 B x spp x pixels sample-buffer read).
"""
import collections
import csv
import json
import os
import shutil
import sys


def sums(path):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        k = "trace_samples" if "trace_samples" in name else "resolve_samples" if "resolve_samples" in name else None
        if k:
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
    return agg


def main():
    src, dst, label = sys.argv[1], sys.argv[2], sys.argv[3]
    os.makedirs(os.path.join(dst, "pmc"), exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "bench_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{label}.csv"))
    out = {}
    for d in ("fetch", "write", "sq", "wait"):
        f = os.path.join(src, d, "bench_counter_collection.csv")
        if os.path.exists(f):
            for (k, c), v in sums(f).items():
                out.setdefault(k, {})[c] = v
    json.dump(out, open(os.path.join(dst, "pmc", f"pmc_sums_{label}.json"), "w"), indent=1)
    t = out["trace_samples"]
    fetch, write = t["FETCH_SIZE"] * 1024 * 2, t["WRITE_SIZE"] * 1024
    r = out["resolve_samples"]
    traffic = {
        "config": "C3", "scaling": "weak", "kernel": "trace_samples", "hbm_bytes_per_launch": fetch + write,
        "fetch_bytes": fetch, "write_bytes": write,
        "resolve_fetch_bytes_check": r["FETCH_SIZE"] * 1024 * 2,
        "valu_lane_utilisation": t.get("SQ_THREAD_CYCLES_VALU", 0) / max(t.get("SQ_ACTIVE_INST_VALU", 1) * 64, 1),
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes over one C3 frame "
                  "(bench.py --steps 1 --warmup 0); KiB; FETCH_SIZE x2 per the gfx950 note in MI355X_MICROARCH.md",
        "source": f"{dst}/pmc/pmc_sums_{label}.json",
    }
    json.dump(traffic, open(os.path.join(os.path.dirname(dst.rstrip("/")), "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
