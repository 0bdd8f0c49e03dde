#!/usr/bin/env python3
"""How many samples a config's fast kernel hands to the replay pass, and the frame time (diagnostic).

    python3 tools/replay_count.py C4[:spp] [C3:100 ...]

Renders each config once with RT_OPT_LAUNCH_LOG on (the library prints, per chunk, the samples the
fast kernel handed over) and then --reps more times, printing the handed-over count per frame, the
rt_render kernel time (fast kernel + replay passes) and the segments."""
import argparse
import os
import re
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(spec, reps):
    import raytracinginoneweekendinrust_amd as rt
    from raytracinginoneweekendinrust_amd.configs import CONFIGS
    name, _, spp = spec.partition(":")
    cfg = CONFIGS[name]
    if spp:
        cfg = cfg.scaled(cfg.width, int(spp))
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    params = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                              seed=cfg.render_seed)
    ds = rt.DeviceScene(scene)
    try:
        times = []
        for i in range(reps + 1):
            _, st = ds.render(cfg.camera(), params)
            times.append(st["kernel_ms"])
            segs = st["segments"]
    finally:
        ds.close()
    return cfg, times, segs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child:  # one config per process: the library's stderr log is read by the parent
        import raytracinginoneweekendinrust_amd as rt
        with rt.options(launch_log=1):
            cfg, times, segs = one(a.configs[0], a.reps)
        print(f"RESULT {a.configs[0]} {statistics.median(times[1:]):.2f} {segs} {cfg.width * cfg.height * cfg.spp}",
              flush=True)
        return
    for spec in a.configs:
        p = subprocess.run([sys.executable, __file__, "--child", "--reps", str(a.reps), spec], capture_output=True,
                           text=True, timeout=600)
        if p.returncode != 0:
            print(p.stdout, p.stderr, file=sys.stderr)
            sys.exit(p.returncode)
        counts = [int(m) for m in re.findall(r"chunk \d+: (\d+) samples replayed", p.stderr)]
        res = [l for l in p.stdout.splitlines() if l.startswith("RESULT")][-1].split()
        frames = a.reps + 1
        print(f"{spec:10s} handed over per frame {sum(counts) / frames:10.1f} (launch log: {counts[:8]}) "
              f"rt_render {res[2]} ms median  segments {res[3]}  samples {res[4]}", flush=True)


if __name__ == "__main__":
    main()
