#!/usr/bin/env python3
"""Per-region wave-cycle profile of trace_samples (diagnostic, GPU box only).

    RT_LIBRARY=raytracinginoneweekendinrust_amd/_lib/librtamd_prof.so \
        python3 tools/region_profile.py [--config C3] [--spp 64]

Renders one frame with the region-instrumented build and prints, per region,
the share of wave cycles, wave executions and the mean active lanes when the
region ran (64 = fully converged). Regions nest: World contains the per-entry
rows (and BVH trips / leaf tests); Finish segment contains Record, Emit and
Scatter; Scatter contains the material rows; materials contain the textures.
The library also prints leaf-box audit records (see kernel.hip LEAF_AUDIT).
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["Refill", "Finish segment", "World", "Record", "Emit", "Scatter", "Marble", "Store", "Checker", "Image",
         "UnitSphere", "Dielectric", "Lambert", "Metal", "Isotropic", "MediumLog"]
COUNT = 52
EXTRA = {44: "BVH loop trip (child tests)", 45: "BVH leaf test", 46: "BVH call setup", 47: "BVH sort + push",
         48: "BVH pop loop", 49: "BVH call total"}
ENTRY0 = 16
# showcase's top-level entries after lowering (lower.cpp merges consecutive top-level spheres into runs)
SHOWCASE = ["boxes BVH", "light rect", "moving sphere", "sphere run (glass, metal, medium boundary)",
            "blue medium", "fog medium", "sphere run (earth, marble)", "spheres BVH (RotY+Tr)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--shard", type=int, default=1, help="render shard 0 of N (bench.py's block interleave)")
    ap.add_argument("--rows", default=None,
                    help="r0:r1 — render only the 8x8-block rows [r0, r1) (rt_prof_rows; the profiling build)")
    ap.add_argument("--bands", type=int, default=0,
                    help="profile the frame in this many bands of block rows, one launch each, and print a "
                         "per-band table (cycles per segment and per-entry shares)")
    args = ap.parse_args()
    if not any(k in os.environ.get("RT_LIBRARY", "") for k in ("_prof", "_audit")):
        sys.exit("set RT_LIBRARY to the _prof or _audit build")
    if args.bands:
        return bands(args)
    import torch
    import raytracinginoneweekendinrust_amd as rt
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import rtopts
    rtopts.apply(rt)
    cfg = rt.CONFIGS[args.config]
    if args.spp:
        cfg = cfg.scaled(cfg.width, args.spp)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    if args.rows:
        import ctypes as C
        from raytracinginoneweekendinrust_amd import _capi
        r0, r1 = (int(v) for v in args.rows.split(":"))
        _capi.lib.rt_prof_rows.argtypes = [C.c_uint32, C.c_uint32]
        assert _capi.lib.rt_prof_rows(r0, r1) == 0
    ds = rt.DeviceScene(scene)
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(), seed=cfg.render_seed,
                         shard_index=0, shard_count=args.shard)
    out = torch.zeros(cfg.width * cfg.height * 3, dtype=torch.float32, device="cuda")
    seg = torch.zeros(1, dtype=torch.int64, device="cuda")
    ds.launch(cfg.camera(), p, out.data_ptr(), seg.data_ptr(), 0)
    torch.cuda.synchronize()
    ms, n = ds.trace_time(reset=True)
    segments = int(seg.item())
    # the library prints its counters on stderr when the scene is freed
    sys.stderr.flush()
    saved = os.dup(2)
    with tempfile.TemporaryFile(mode="w+") as tf:
        os.dup2(tf.fileno(), 2)
        ds.close()
        os.dup2(saved, 2)
        tf.seek(0)
        captured = tf.read().splitlines()
        lines = [ln for ln in captured if ln.startswith('{"rt_profile"')]
        for ln in captured:
            if ln.startswith(('{"leaf_audit', '{"audit', '{"trav_audit', '{"bounds_audit', '{"trips_hist', '{"wave_times', '{"tp_gseg', '{"role_ev')):
                print(ln)
    if not lines:  # an audit build: no region counters
        return
    v = json.loads(lines[-1])["rt_profile"]
    cyc, cnt, lanes = v[:COUNT], v[COUNT:2 * COUNT], v[2 * COUNT:]
    total = cyc[0] + cyc[1] + cyc[2]  # refill + finish_segment + world_hit: the whole loop
    samples = cfg.width * cfg.height * cfg.spp // args.shard
    print(f"{cfg.name} {cfg.width}x{cfg.height} {cfg.spp}spp: trace {ms:.1f} ms, {segments} segments, "
          f"{segments / samples:.3f} seg/sample, wave cycles refill+segment = {total:.4g}")
    rows = []
    for i in range(COUNT):
        if cnt[i] == 0:
            continue
        name = EXTRA[i] if i in EXTRA else NAMES[i] if i < ENTRY0 else (f"entry {i - ENTRY0}: " + (SHOWCASE[i - ENTRY0] if cfg.scene == "showcase"
                                                                        and i - ENTRY0 < len(SHOWCASE) else ""))
        rows.append((name, cyc[i] / total, cnt[i], lanes[i] / cnt[i], cyc[i] / cnt[i]))
    print(f"{'region':34s} {'cyc%':>7s} {'wave-execs':>12s} {'lanes':>6s} {'cyc/exec':>9s}")
    for name, frac, c, ln, ce in rows:
        print(f"{name:34s} {100 * frac:7.2f} {c:12d} {ln:6.1f} {ce:9.0f}")
    print(json.dumps({"band": args.rows, "trace_ms": ms, "segments": segments, "wave_cycles": total,
                      "regions": {name: {"cyc": cyc[i], "execs": cnt[i], "lanes": lanes[i]}
                                  for i, name in enumerate(_names(cfg)) if cnt[i]}}))


def _names(cfg):
    out = []
    for i in range(COUNT):
        out.append(EXTRA[i] if i in EXTRA else NAMES[i] if i < ENTRY0 else (
            f"entry {i - ENTRY0}: " + (SHOWCASE[i - ENTRY0] if cfg.scene == "showcase" and i - ENTRY0 < len(SHOWCASE)
                                       else "")))
    return out


def bands(args):
    """One launch per band of 8x8-block rows (a process each: the library's counters accumulate for
    the process), then per band: wave cycles per segment and the per-region cycles per segment."""
    import subprocess
    sys.path.insert(0, ROOT)
    from raytracinginoneweekendinrust_amd.configs import CONFIGS
    cfg = CONFIGS[args.config]
    rows_total = (cfg.height + 7) // 8
    edges = [round(i * rows_total / args.bands) for i in range(args.bands + 1)]
    res = []
    for b in range(args.bands):
        cmd = [sys.executable, os.path.abspath(__file__), "--config", args.config, "--rows", f"{edges[b]}:{edges[b + 1]}"]
        if args.spp:
            cmd += ["--spp", str(args.spp)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            sys.exit(r.stderr[-2000:])
        line = [ln for ln in r.stdout.splitlines() if ln.startswith('{"band"')][-1]
        res.append(json.loads(line))
        print(r.stdout, flush=True)
    keys = [k for k in res[0]["regions"] if k.startswith("entry") or k.startswith("BVH") or k in
            ("Refill", "Record", "Marble", "UnitSphere", "MediumLog", "Scatter")]
    print(f"{'rows':>9s} {'segs':>11s} {'cyc/seg':>8s} " + " ".join(f"{k[:12]:>12s}" for k in keys))
    for r in res:
        segs = max(r["segments"], 1)
        print(f"{r['band']:>9s} {r['segments']:11d} {r['wave_cycles'] / segs:8.0f} " +
              " ".join(f"{r['regions'].get(k, {}).get('cyc', 0) / segs:12.0f}" for k in keys))
    print(json.dumps({"bands": res}))


if __name__ == "__main__":
    main()
