#!/usr/bin/env python3
"""One rank's share of the multi-GPU bench, timed on device 0 (diagnostic): the trace time of
shard r of N (8x8 blocks b % N == r, bench.py's strong-scaling decomposition) of a config,
to see what an N-GPU step costs each GPU before the gather.

    python3 tools/shard_time.py --config C3 --n 8 [--rank 0] [--reps 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--spp", type=int, default=None, help="override the config's samples per pixel")
    ap.add_argument("--shard-only", action="store_true", help="skip the whole-frame (1-rank) reference run")
    ap.add_argument("--pipeline", action="store_true",
                    help="frames in flight (bench.py --pipeline on): rotate scene handles and streams "
                         "and report the steady-state time per step")
    ap.add_argument("--handles", type=int, default=3, help="scene handles (and streams) in rotation with --pipeline")
    ap.add_argument("--stream-replay", action="store_true",
                    help="with --pipeline: keep the streaming replay pass (no RT_FLAG_FRAMES_IN_FLIGHT)")
    a = ap.parse_args()
    import torch
    import raytracinginoneweekendinrust_amd as rt
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import rtopts
    rtopts.apply(rt)  # RT_GROUP=... of the session scripts
    cfg = rt.CONFIGS[a.config]
    if a.spp:
        cfg = cfg.scaled(cfg.width, a.spp)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    ds = rt.DeviceScene(scene)
    out = torch.zeros(cfg.width * cfg.height * 3, dtype=torch.float32, device="cuda")
    if a.pipeline:
        nh = max(2, a.handles)
        dss = [ds] + [rt.DeviceScene(scene) for _ in range(nh - 1)]
        outs = [out] + [torch.zeros_like(out) for _ in range(nh - 1)]
        st = [torch.cuda.Stream() for _ in range(nh)]
        for n in ([a.n] if a.shard_only else sorted({1, a.n})):
            p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                                 seed=cfg.render_seed, shard_index=a.rank if n > 1 else 0, shard_count=n,
                                 frames_in_flight=not a.stream_replay)
            for k in range(nh):  # warm-up
                dss[k].launch(cfg.camera(), p, outs[k].data_ptr(), 0, st[k].cuda_stream)
            torch.cuda.synchronize()
            import time
            t0 = time.perf_counter()
            for k in range(a.reps):
                dss[k % nh].launch(cfg.camera(), p, outs[k % nh].data_ptr(), 0, st[k % nh].cuda_stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.reps
            print(f"{cfg.name} shard {a.rank if n > 1 else 0}/{n}: pipelined step {ms:.2f} ms "
                  f"({a.reps} frames, {nh} handles)", flush=True)
        for d in dss:
            d.close()
        return
    for n in ([a.n] if a.shard_only else sorted({1, a.n})):
        p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                             seed=cfg.render_seed, shard_index=a.rank if n > 1 else 0, shard_count=n)
        ds.launch(cfg.camera(), p, out.data_ptr(), 0, 0)  # warm-up
        torch.cuda.synchronize()
        ds.trace_time(reset=True)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(a.reps):
            ds.launch(cfg.camera(), p, out.data_ptr(), 0, 0)
        ev1.record()
        torch.cuda.synchronize()
        ms, launches = ds.trace_time(reset=True)
        print(f"{cfg.name} shard {a.rank if n > 1 else 0}/{n}: step {ev0.elapsed_time(ev1) / a.reps:.2f} ms, "
              f"trace kernel {ms / max(launches, 1):.2f} ms", flush=True)
    ds.close()


if __name__ == "__main__":
    main()
