#!/usr/bin/env python3
"""bench.py — throughput of the MI355X path-tracing hot path on BASELINE's headline workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one render launch of the C3 frame (showcase, 1200x800, 500 spp,
depth 50) with the scene already resident in HBM. Weak scaling (default): every
rank renders the full frame with its own disjoint sample range
(sample_base = rank * spp), i.e. N ranks together produce an N*500-spp
progressive render; no collective touches the data path. Strong scaling
(--scaling strong) interleaves 8x8 blocks across ranks instead.

Prints ONE JSON line on rank 0 (metric/value/unit, roofline, cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "Msamples/s (rays traced/s) + HBM GB/s vs roofline, showcase@1200x800x500spp"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters"

# Algorithmic bytes per unit: 32 B per BVH node visit, per-primitive
# record sizes, 32 B material record per hit, 3 B per image texel, 12 B framebuffer per pixel.
BYTES = {"node_visits": 32, "sphere_tests": 20, "msphere_tests": 36, "rect_tests": 28, "tri_tests": 40,
         "medium_tests": 12, "hits": 32, "texel_fetches": 3}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def bytes_per_sample(counters: dict, spp: int) -> float:
    """Algorithmic bytes per camera sample of trace_samples: the scene records the
    reference algorithm touches (counted by the oracle) + the 12-byte radiance
    record each sample writes to the HBM sample buffer + 12/spp framebuffer."""
    total = sum(BYTES[k] * counters[k] for k in BYTES)
    return total / counters["samples"] + 12.0 + 12.0 / spp


def cpu_threads() -> int:
    n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, n)


SUBSAMPLE = 64  # counts from a fixed 1/64 subsample at the config's spp and depth


def oracle_measure(cfg, scene, threads: int):
    """Oracle render of the fixed 1/64 block subsample (8x8 blocks b with
    b % 64 == 21, spread over the whole frame) at full spp/depth: the CPU baseline
    (Msamples/s on `threads` host threads) and the reference algorithm's per-sample
    counts for the roofline's algorithmic bytes."""
    import oracle_ffi as orc
    import raytracinginoneweekendinrust_amd as rt
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(), shard_index=21,
                         shard_count=SUBSAMPLE, seed=cfg.render_seed)
    _, cnt = orc.render(scene, cfg.camera(), p, threads=threads)
    return cnt


def rank_work(rt, cfg, rank: int, world: int, scaling: str, exact_bvh: bool = False):
    """The multi-GPU decomposition: render params of `rank` and its
    pixel count. weak: every rank renders the whole frame with samples
    [rank*spp, (rank+1)*spp); strong: 8x8 blocks b with b % world == rank."""
    W, H, spp = cfg.width, cfg.height, cfg.spp
    if scaling == "weak":
        params = rt.render_params(W, H, spp, cfg.depth, background=cfg.background(), seed=cfg.render_seed,
                                  sample_base=rank * spp, exact_bvh=exact_bvh)
        return params, W * H
    params = rt.render_params(W, H, spp, cfg.depth, background=cfg.background(), seed=cfg.render_seed,
                              shard_index=rank, shard_count=world, exact_bvh=exact_bvh)
    bx, by = (W + 7) // 8, (H + 7) // 8
    pixels = 0
    for b in range(rank, bx * by, world):
        x0, y0 = (b % bx) * 8, (b // bx) * 8
        pixels += (min(W, x0 + 8) - x0) * (min(H, y0 + 8) - y0)
    return params, pixels


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--exact-bvh", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist

    import raytracinginoneweekendinrust_amd as rt

    if not torch.cuda.is_available():
        log("bench.py needs a GPU (the HIP path has no CPU fallback)")
        return 2
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world)  # RCCL: barrier + max-reduce of timings only

    cfg = rt.CONFIGS[args.config]
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    ds = rt.DeviceScene(scene, device=local_rank)
    cam = cfg.camera()
    W, H, spp = cfg.width, cfg.height, cfg.spp
    params, pixels_rank = rank_work(rt, cfg, rank, world, args.scaling, args.exact_bvh)
    out = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    seg = torch.zeros(1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        ds.launch(cam, params, out.data_ptr(), seg.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ds.trace_time(reset=True)  # drop warmup launches from the per-launch timing
    seg.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps          # device time of a whole step (all kernels)
    trace_total_ms, trace_launches = ds.trace_time(reset=True)  # HIP events around each trace_samples launch
    kernel_ms = trace_total_ms / max(trace_launches, 1)
    segments = int(seg.item())
    t = torch.tensor([wall, float(segments)], dtype=torch.float64, device="cuda")
    if world > 1:
        tw = t[:1].clone()
        dist.all_reduce(tw, op=dist.ReduceOp.MAX)
        ts = t[1:].clone()
        dist.all_reduce(ts, op=dist.ReduceOp.SUM)
        wall_max, seg_total = float(tw.item()), float(ts.item())
    else:
        wall_max, seg_total = wall, float(segments)
    samples_rank_launch = pixels_rank * spp
    total_samples = (samples_rank_launch * world if args.scaling == "weak" else W * H * spp) * args.steps
    img_ok = bool(torch.isfinite(out).all().item())

    if rank == 0:
        threads = cpu_threads()
        cpu = None
        try:
            cnt = oracle_measure(cfg, scene, threads)
            if world == 1 and not args.no_cpu_baseline:
                cpu = {"value": cnt["samples"] / cnt["seconds"] / 1e6, "unit": "Msamples/s", "cores": cnt["threads"],
                       "kind": "port",
                       "sample": f"{cfg.name} 8x8 blocks b % {SUBSAMPLE} == 21 ({cnt['samples'] // spp} px, 1/64 of "
                                 f"the frame) at {spp} spp depth {cfg.depth}: {cnt['samples']} samples in "
                                 f"{cnt['seconds']:.1f}s (C oracle, pthreads)"}
        except Exception as e:  # the oracle is optional on the box; the product path is not
            log(f"oracle unavailable: {e}")
            cnt = None
        b_sample = bytes_per_sample(cnt, spp) if cnt else None
        samples_per_trace_launch = samples_rank_launch * args.steps / max(trace_launches, 1)
        achieved = (b_sample * samples_per_trace_launch / (kernel_ms / 1e3) / 1e9) if b_sample else None
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                j = json.load(open(pmc))
                if j.get("config") == cfg.name and j.get("scaling", "weak") == args.scaling:
                    traffic = j.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        value = total_samples / wall_max / 1e6
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene generator, src/main.rs:559-686 restated)",
            "config": {"workload": f"{cfg.name} {cfg.scene} {W}x{H} {spp}spp depth {cfg.depth}",
                       "scene": cfg.scene, "width": W, "height": H, "spp": spp, "max_depth": cfg.depth,
                       "parallelism": ("weak: full frame per GPU, disjoint sample ranges" if args.scaling == "weak"
                                       else "strong: 8x8 blocks interleaved across GPUs"),
                       "exact_bvh": args.exact_bvh},
            "rays_per_s": seg_total / wall_max,
            "segments_per_sample": seg_total / total_samples if total_samples else None,
            "image_finite": img_ok,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                         "kernel": "trace_samples", "kernel_ms": kernel_ms, "launches_per_step":
                             trace_launches / args.steps, "step_device_ms": step_ms,
                         "bytes_per_sample": b_sample, "samples_per_launch": samples_per_trace_launch},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ds.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
