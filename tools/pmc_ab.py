#!/usr/bin/env python3
"""HBM traffic per frame of A/B variants (diagnostic).

    python3 tools/pmc_ab.py <dir> [<dir> ...]

Each <dir> holds two rocprofv3 runs of `tools/ab_time.py --reps 1 <one lib spec>` (two frames:
the warm-up and the timed one), `fetch/` with `--pmc FETCH_SIZE` and `write/` with
`--pmc WRITE_SIZE` (tools/sessions/r06/r06_sess8.sh). Every trace_samples dispatch is summed and
divided by the number of fast-kernel dispatches (trace_samples<0, ...>: one per frame at the
spp these runs use), so a frame's streaming replay pass counts with it. FETCH_SIZE and
WRITE_SIZE are KiB per dispatch; FETCH_SIZE is doubled on gfx950 (MI355X_MICROARCH.md, the
HBM/rocprofv3 section), as tools/valu_roofline.py does.
"""
import collections
import csv
import glob
import os
import sys


def per_frame(run_dir, counter):
    total, fast = 0.0, set()
    for path in glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if "trace_samples" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            total += float(r["Counter_Value"])
            if "trace_samples<0," in r["Kernel_Name"]:
                fast.add(r["Dispatch_Id"])
    return (total * 1024.0 / len(fast), len(fast)) if fast else (None, 0)


def main():
    rows = collections.OrderedDict()
    for d in sys.argv[1:]:
        fetch, nf = per_frame(os.path.join(d, "fetch"), "FETCH_SIZE")
        write, nw = per_frame(os.path.join(d, "write"), "WRITE_SIZE")
        rows[d] = (None if fetch is None else 2.0 * fetch, write, nf, nw)
    print(f"{'variant':48s} {'fetch GB':>9s} {'write GB':>9s} {'HBM GB':>9s}  frames")
    for d, (f, w, nf, nw) in rows.items():
        hbm = None if f is None or w is None else f + w
        fmt = lambda v: f"{v / 1e9:9.2f}" if v is not None else f"{'-':>9s}"
        print(f"{os.path.basename(d.rstrip('/')):48s} {fmt(f)} {fmt(w)} {fmt(hbm)}  {nf}/{nw}")


if __name__ == "__main__":
    main()
