#!/usr/bin/env python3
"""Attribute the C3 throughput dip to regions (diagnostic; reads tools/region_profile.py --bands output).

    python3 tools/dip_attribution.py gpurun_out/r06_s5/bands.log [--dip 50:70]

Each band of 8x8-block rows was rendered alone (rt_prof_rows) by the region-profiling build. The
pool takes blocks last first, i.e. the top block rows first, so the launch's time axis runs from
band 90:100 down to band 0:10; the dip of the throughput histogram (tp_gseg_per_s) is the stretch
whose segments cost the most wave cycles. Per band: wave cycles per segment in total and per
region; then, for the dip bands against the rest of the frame (segment-weighted), the extra wave
cycles per segment and the share of that extra each region accounts for. Regions are the
profiler's top-level ones (Refill, the eight top-level entries of showcase's list walk, and the
shading steps outside the walk: Record, Marble); the BVH rows are shown separately as the
breakdown of entries 0 and 7 (their cycles are inside those entries)."""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--dip", default="50:70", help="block rows of the dip, r0:r1 (bands inside it)")
    a = ap.parse_args()
    bands = None
    for line in open(a.log):
        if line.startswith('{"bands"'):
            bands = json.loads(line)["bands"]
    assert bands, "no band summary in the log"
    d0, d1 = (int(v) for v in a.dip.split(":"))
    top = [k for k in bands[0]["regions"] if k == "Refill" or k.startswith("entry ") or k in ("Record", "Marble")]
    bvh = [k for k in bands[0]["regions"] if k.startswith("BVH")]

    def per_seg(rows, key):
        segs = sum(r["segments"] for r in rows)
        return sum(r["regions"].get(key, {}).get("cyc", 0) for r in rows) / max(segs, 1)

    def total(rows):
        segs = sum(r["segments"] for r in rows)
        return sum(sum(r["regions"].get(k, {}).get("cyc", 0) for k in top) for r in rows) / max(segs, 1)

    print(f"{'band':>8s} {'segments':>11s} {'cyc/seg':>8s} " + " ".join(f"{k.split(':')[0][:9]:>9s}" for k in top))
    for r in bands:
        print(f"{r['band']:>8s} {r['segments']:11d} {total([r]):8.0f} " + " ".join(f"{per_seg([r], k):9.0f}" for k in top))
    dip = [r for r in bands if d0 <= int(r["band"].split(":")[0]) and int(r["band"].split(":")[1]) <= d1]
    rest = [r for r in bands if r not in dip]
    extra = total(dip) - total(rest)
    print(f"\ndip rows {a.dip}: {total(dip):.0f} wave cycles per segment, rest of the frame {total(rest):.0f}: "
          f"+{extra:.0f} ({100 * extra / total(rest):.0f}%)")
    print(f"{'region':40s} {'dip':>7s} {'rest':>7s} {'extra':>7s} {'share':>6s}")
    rows = sorted(((k, per_seg(dip, k), per_seg(rest, k)) for k in top), key=lambda x: -(x[1] - x[2]))
    for k, dv, rv in rows:
        print(f"{k:40s} {dv:7.0f} {rv:7.0f} {dv - rv:+7.0f} {100 * (dv - rv) / extra:5.1f}%")
    print("\ninside the BVH entries (0 and 7):")
    for k in bvh:
        dv, rv = per_seg(dip, k), per_seg(rest, k)
        lanes_d = sum(r["regions"].get(k, {}).get("lanes", 0) for r in dip) / max(
            sum(r["regions"].get(k, {}).get("execs", 0) for r in dip), 1)
        lanes_r = sum(r["regions"].get(k, {}).get("lanes", 0) for r in rest) / max(
            sum(r["regions"].get(k, {}).get("execs", 0) for r in rest), 1)
        print(f"{k:40s} {dv:7.0f} {rv:7.0f} {dv - rv:+7.0f}  lanes {lanes_d:5.1f} vs {lanes_r:5.1f}")


if __name__ == "__main__":
    main()
