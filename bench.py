#!/usr/bin/env python3
"""bench.py — throughput of the MI355X path-tracing hot path on BASELINE's headline workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one whole C3 frame (showcase, 1200x800, 500 spp, depth 50) with the
scene already resident in HBM. At N GPUs (one process each) the
frame is fixed (strong scaling, the north-star workload): rank r renders the 8x8
blocks b % N == r and the shards are gathered to rank 0 INSIDE the timed region
(frame_gather.FrameGather: every rank packs its blocks with rt_shard_pack, one gloo
barrier, and rank 0 pulls the other ranks' packed shards straight out of their
IPC-mapped device buffers over xGMI with rt_shard_pull_unpack; the /dev/shm bounce is
the fallback where IPC is refused) — the composite of src/renderer.rs:63-95. No collective touches the data path; gloo carries only the
barriers and the max over ranks of the timings. `--scaling weak` (opt-in) renders
the full frame on every rank with disjoint sample ranges instead.

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
# rows shared by every workgroup, served by each XCD's L2: 16.8-18.8 TB/s chip-wide (the top of the range),
# MI355X_MICROARCH.md "Indexed rows: gather into LDS"
L2_PEAK_GBS = 18800.0

# Algorithmic bytes per unit: 32 B per BVH node visit, per-primitive
# record sizes, 32 B material record per hit, 3 B per image texel, 12 B framebuffer per pixel.
BYTES = {"node_visits": 32, "sphere_tests": 20, "msphere_tests": 36, "rect_tests": 28, "tri_tests": 40,
         "medium_tests": 12, "hits": 32, "texel_fetches": 3}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


IMPL_BYTES_PER_SAMPLE = 12.0  # the implementation's own sample-buffer record (written once, read once): not §8(d)


def bytes_per_sample(counters: dict, spp: int) -> float:
    """Algorithmic bytes per camera sample exactly as SURVEY.md §8(d) states them: the scene
    records the reference algorithm touches (counted by the oracle's instrumented recursion)
    + 12/spp framebuffer. The implementation's 12-byte sample-buffer record is NOT part of
    it (reported apart as `impl_bytes_per_sample`)."""
    total = sum(BYTES[k] * counters[k] for k in BYTES)
    return total / counters["samples"] + 12.0 / spp


ISSUE_CEILING_TOL = 0.15  # roofline.bound = "valu" when the PMC issue fraction is within 15% of its ceiling


def roofline_bound(valu) -> tuple:
    """The kernel's bound as the committed PMC for this very library shows it: "valu" when the
    SIMDs issue VALU in at least 85% of the quad-cycles the measured ceiling allows (the kernel
    is then issue-bound, whatever its HBM rate), else "latency"; "hbm" (§8(d)'s nominal bound)
    only when no PMC summary matches the loaded library."""
    if not valu or valu.get("issue_quads") is None:
        return "hbm", "no PMC summary for this library: §8(d)'s nominal HBM bound"
    q, ceil = float(valu["issue_quads"]), float(valu.get("issue_quads_ceiling") or 0.94)
    if q >= (1.0 - ISSUE_CEILING_TOL) * ceil:
        return "valu", f"PMC: VALU issue in {q:.3f} of the quad-cycles, ceiling {ceil} (within 15%)"
    return "latency", f"PMC: VALU issue {q:.3f} of the quad-cycles, below 85% of the {ceil} ceiling (waits dominate)"


def host_nproc() -> int:
    """The CPUs this process may run on (its affinity mask: what `nproc` prints, without
    starting a program from a GPU-initialised process)."""
    return len(os.sched_getaffinity(0))


def cpu_share():
    """The CPU time this process's cgroup may use, in CPUs (cgroup v2 cpu.max or v1
    cfs_quota/cfs_period), and where it was read; (None, reason) without a quota."""
    paths = ["/sys/fs/cgroup/cpu.max"]
    try:  # cgroup v2: this process's own group first ("0::/path" in /proc/self/cgroup)
        for line in open("/proc/self/cgroup"):
            if line.startswith("0::"):
                paths.insert(0, "/sys/fs/cgroup" + line.strip()[3:].rstrip("/") + "/cpu.max")
    except Exception:
        pass
    for path in paths:
        try:
            quota, period = open(path).read().split()[:2]
            if quota == "max":
                return None, f"{path}: max (no quota)"
            return int(quota) / int(period), f"{path}: {quota} {period}"
        except Exception:
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per, f"cpu.cfs_quota_us {q} / cpu.cfs_period_us {per}"
        return None, "cpu.cfs_quota_us -1 (no quota)"
    except Exception:
        return None, "no cgroup cpu quota readable"


def cpu_threads() -> int:
    """Threads for the CPU baseline: every CPU of the affinity mask, capped by OMP_NUM_THREADS where the
    launcher sets the box's CPU share (16 per GPU on the GPU pool, whose nproc shows the whole host)."""
    n = host_nproc()
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, n)


PMC_DIRS = tuple(os.path.join(ROOT, "profiles", d) for d in ("r06", "r05", "r04", "r03", ""))


def library_md5() -> str:
    """md5 of the librtamd.so this process loaded (the PMC summaries record the one they profiled)."""
    import hashlib

    from raytracinginoneweekendinrust_amd import _capi
    with open(_capi.LIB_PATH, "rb") as f:
        return hashlib.md5(f.read()).hexdigest()


def pmc_summary(kind: str, cfg_name: str, md5: str):
    """A committed PMC summary (tools/valu_roofline.py: kind 'valu' or 'traffic') of `cfg_name`'s
    trace kernel, or None. Only a summary that records the md5 of the very library this process
    loaded counts: after any rebuild without a re-profile the line carries null, not stale counters."""
    for d in PMC_DIRS:
        for name in (f"pmc_{kind}_{cfg_name}.json", f"pmc_{kind}.json"):
            try:
                j = json.load(open(os.path.join(d, name)))
            except Exception:
                continue
            if j.get("config") == cfg_name and j.get("library_md5") == md5:
                return j
    return None


SUBSAMPLE = 64  # counts from a fixed 1/64 subsample at the config's spp and depth


def oracle_measure(cfg, scene, threads: int, full: bool = False):
    """Oracle render of the fixed 1/64 block subsample (8x8 blocks b with
    b % 64 == 21, spread over the whole frame) at full spp/depth, or of the whole frame
    (`full`): the CPU baseline (Msamples/s on `threads` host threads) and the reference
    algorithm's per-sample counts for the roofline's algorithmic bytes."""
    import oracle_ffi as orc
    import raytracinginoneweekendinrust_amd as rt
    shard = {} if full else {"shard_index": 21, "shard_count": SUBSAMPLE}
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(),
                         seed=cfg.render_seed, **shard)
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
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="oracle threads for cpu_baseline (default: the box's CPU share; C1: 1, as BASELINE config 1 "
                         "states, over the whole frame)")
    ap.add_argument("--exact-bvh", action="store_true")
    ap.add_argument("--gather", choices=["auto", "ipc", "shm"], default="auto",
                    help="N>1 frame gather transport (frame_gather.FrameGather)")
    ap.add_argument("--pipeline", choices=["auto", "on", "off"], default="auto",
                    help="frames in flight per rank (three scene handles and streams, RT_FLAG_FRAMES_IN_FLIGHT): "
                         "frame k+1's trace kernel takes the SIMDs frame k's last paths leave, and frame k is "
                         "gathered while frame k+1 renders; auto = on for N>1 (strong scaling), off for one GPU")
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
    # one GPU per rank; with fewer GPUs than ranks (a rehearsal on a one-GPU box) ranks share them
    ndev = torch.cuda.device_count()
    if local_rank >= ndev:
        log(f"note: LOCAL_RANK {local_rank} >= {ndev} GPUs; rank shares GPU {local_rank % ndev}")
    local_rank = local_rank % ndev
    torch.cuda.set_device(local_rank)
    if world > 1:  # gloo on the host: barriers and the max over ranks only; no collective on the data path
        dist.init_process_group("gloo", rank=rank, world_size=world)

    cfg = rt.CONFIGS[args.config]
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    cam = cfg.camera()
    W, H, spp = cfg.width, cfg.height, cfg.spp
    params, pixels_rank = rank_work(rt, cfg, rank, world, args.scaling, args.exact_bvh)
    pipeline = args.pipeline == "on" or (args.pipeline == "auto" and world > 1)
    # Three handles: a handle's launch waits for its previous one, whose replay and resolve kernels get
    # SIMDs only in the next launch's drain. One rank of 8 on C3: serial 55.9 ms, two handles 55.3, three
    # with the flag 54.6 (profiles/r05/shard/c3_rank_of_8_frames_in_flight.log).
    nbuf = 3 if pipeline else 1
    if pipeline:
        params.flags |= rt._capi.RT_FLAG_FRAMES_IN_FLIGHT
    # one scene handle per frame in flight (each serialises its own launches and owns its sample buffer)
    dss = [rt.DeviceScene(scene, device=local_rank) for _ in range(nbuf)]
    outs = [torch.zeros(W * H * 3, dtype=torch.float32, device="cuda") for _ in range(nbuf)]
    segs = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(nbuf)]
    streams = [torch.cuda.Stream() for _ in range(nbuf)] if pipeline else [torch.cuda.current_stream()]
    stream = streams[0]
    gather = None
    if args.scaling == "strong" and world > 1:
        from raytracinginoneweekendinrust_amd.frame_gather import FrameGather
        gather = FrameGather(W, H, rank, world, device=f"cuda:{local_rank}", transport=args.gather)
    frame = [outs[0]]
    state = {"k": 0, "pending": None}

    def finish(h):  # gather frame slot h (rank 0 ends holding the whole frame), ordered after its render
        if gather is not None:
            with torch.cuda.stream(streams[h]):
                frame[0] = gather.gather(outs[h])
        else:
            frame[0] = outs[h]

    def step():
        # render this step's frame; pipelined, the previous step's frame is gathered while it renders
        h = state["k"] % nbuf
        state["k"] += 1
        dss[h].launch(cam, params, outs[h].data_ptr(), segs[h].data_ptr(), streams[h].cuda_stream)
        if pipeline:
            if state["pending"] is not None:
                finish(state["pending"])
            state["pending"] = h
        else:
            finish(h)

    def flush():  # the last frame in flight
        if state["pending"] is not None:
            finish(state["pending"])
            state["pending"] = None

    for _ in range(args.warmup):
        step()
    flush()
    torch.cuda.synchronize()
    for d in dss:
        d.trace_time(reset=True)  # drop warmup launches from the per-launch timing
    for sg in segs:
        sg.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    flush()
    if pipeline:
        for st_ in streams[1:]:
            stream.wait_stream(st_)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps          # device time of a whole step (all kernels)
    trace_total_ms, trace_launches = 0.0, 0
    for d in dss:  # HIP events around each trace_samples launch
        ms_, n_ = d.trace_time(reset=True)
        trace_total_ms += ms_
        trace_launches += n_
    kernel_ms = trace_total_ms / max(trace_launches, 1)
    segments = int(sum(int(sg.item()) for sg in segs))
    t = torch.tensor([wall, float(segments)], dtype=torch.float64)
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
    img_ok = bool(torch.isfinite(frame[0]).all().item()) if frame[0] is not None else None
    frame_sum = float(frame[0].double().sum().item()) if rank == 0 and frame[0] is not None else None
    frame_md5 = None
    if rank == 0 and frame[0] is not None:  # position-sensitive: the frame's bytes, not a sum over them
        import hashlib
        frame_md5 = hashlib.md5(frame[0].cpu().numpy().tobytes()).hexdigest()

    if rank == 0:
        # BASELINE.json config 1 (C1) is the single-thread CPU reference over the whole frame
        c1 = cfg.name == "C1" and args.cpu_threads is None
        threads = 1 if c1 else (args.cpu_threads or cpu_threads())
        cpu = None
        try:
            cnt = oracle_measure(cfg, scene, threads, full=c1)
            if world == 1 and not args.no_cpu_baseline:
                v = cnt["samples"] / cnt["seconds"] / 1e6
                share, share_src = cpu_share()
                nproc = host_nproc()
                cpu = {"value": v, "unit": "Msamples/s", "cores": cnt["threads"],
                       "kind": "port", "label": "oracle restatement (C, pthreads)", "host_nproc": nproc,
                       "cpu_quota_cpus": share, "cpu_quota_source": share_src,
                       "per_core": v / cnt["threads"],
                       # rayon's par_iter over every logical CPU (src/renderer.rs:63-85) on the whole host:
                       # NOT measured (the box grants this process `cpu_quota_cpus` CPUs of CPU time, and
                       # the pool asks for worker pools sized to that share); the per-thread rate times
                       # host_nproc, i.e. perfect linear scaling, an upper bound for the reference's CPU path
                       "host_nproc_linear_extrapolation": v / cnt["threads"] * nproc,
                       "note": "the C oracle restatement of the reference (oracle/oracle.c), the Rust reference "
                               "cannot be built here; threads = the affinity mask capped by OMP_NUM_THREADS "
                               "(the box's CPU share, see cpu_quota_cpus); host_nproc_linear_extrapolation is "
                               "per_core x host_nproc, not a measurement",
                       "sample": (f"{cfg.name} whole frame ({cnt['samples'] // spp} px)" if c1 else
                                  f"{cfg.name} 8x8 blocks b % {SUBSAMPLE} == 21 ({cnt['samples'] // spp} px, 1/64 of "
                                  f"the frame)") + f" at {spp} spp depth {cfg.depth}: {cnt['samples']} samples in "
                                 f"{cnt['seconds']:.1f}s (C oracle, {cnt['threads']} thread(s))"}
        except Exception as e:  # the oracle is optional on the box; the product path is not
            log(f"oracle unavailable: {e}")
            cnt = None
        b_sample = bytes_per_sample(cnt, spp) if cnt else None
        samples_per_trace_launch = samples_rank_launch * args.steps / max(trace_launches, 1)
        achieved = (b_sample * samples_per_trace_launch / (kernel_ms / 1e3) / 1e9) if b_sample else None
        md5 = library_md5()
        tj = pmc_summary("traffic", cfg.name, md5) if world == 1 else None
        traffic = tj.get("hbm_bytes_per_launch") if tj else None
        valu = pmc_summary("valu", cfg.name, md5) if world == 1 else None
        if valu:
            valu = {k: v for k, v in valu.items() if k != "counters"}
        value = total_samples / wall_max / 1e6
        bound, bound_why = roofline_bound(valu)
        traffic_gbs = (traffic / (kernel_ms / 1e3) / 1e9) if traffic else None
        if cpu:
            cpu["gpu_over_cpu"] = value / cpu["value"]
            cpu["gpu_over_host_nproc_extrapolation"] = value / cpu["host_nproc_linear_extrapolation"]
        line = {
            # BASELINE.json's metric is quoted on C3; the other configs name their own workload
            "metric": METRIC if cfg.name == "C3" else
            f"Msamples/s (rays traced/s) + HBM GB/s vs roofline, {cfg.scene}@{W}x{H}x{spp}spp",
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
                                       else f"strong: one fixed frame, 8x8 blocks b % {world} == rank per GPU, shards "
                                            "gathered to rank 0 inside the timed region (rt_shard_pack on every rank, "
                                            "then rank 0 pulls the peers' IPC-mapped shards over xGMI with "
                                            "rt_shard_pull_unpack, or the /dev/shm bounce; no collective)" if world > 1
                                       else "one GPU: the whole frame"),
                       "gather": gather.transport if gather is not None else None,
                       "pipeline": ("frames in flight per rank: frame k+1 renders on the next of three scene "
                                    "handles and streams while frame k drains and is gathered "
                                    "(RT_FLAG_FRAMES_IN_FLIGHT); every frame is complete and gathered inside the "
                                    "timed region" if pipeline else None),
                       "exact_bvh": args.exact_bvh},
            "rays_per_s": seg_total / wall_max,
            "segments": int(seg_total),
            "segments_per_sample": seg_total / total_samples if total_samples else None,
            "image_finite": img_ok,
            "frame_sum": frame_sum,
            "frame_md5": frame_md5,
            "roofline": {"bound": bound, "bound_source": bound_why,
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                         # the same rate against the XCD L2's measured shared-row rate (the scene's home)
                         "l2_peak": L2_PEAK_GBS, "l2_frac": (achieved / L2_PEAK_GBS) if achieved else None,
                         "achieved_is": "SURVEY.md §8(d) algorithmic bytes per sample (the reference algorithm's "
                                        "scene reads, counted by the oracle, + 12/spp framebuffer) x samples / "
                                        "trace-kernel time: an L2 scene-read rate (the scene is L2-resident), "
                                        "priced against HBM peak as §8(d) asks; the kernel's measured limit is in "
                                        "`bound` / `valu` (vector-ALU issue against the measured ceiling), and its "
                                        "real HBM use in `hbm_frac`",
                         "traffic_GBs": traffic_gbs,
                         # measured memory-side bytes (PMC) per launch / kernel time, against HBM peak
                         "hbm_frac": (traffic_gbs / HBM_PEAK_GBS) if traffic_gbs else None,
                         "valu": valu,
                         "pmc_library_md5": md5,
                         "kernel": "trace_samples", "kernel_ms": kernel_ms,
                         # pipelined (N > 1): a launch's HIP events span the neighbouring frames' launches on
                         # the other handles, so kernel_ms and the rates above are overlapped spans, not
                         # comparable with the one-GPU line
                         "kernel_ms_is": ("overlapped: frames in flight, each launch's events span the "
                                          "concurrent launches on the other handles" if pipeline else
                                          "per trace launch: HIP events on the launch stream"),
                         "launches_per_step": trace_launches / args.steps, "step_device_ms": step_ms,
                         "bytes_per_sample": b_sample, "impl_bytes_per_sample": IMPL_BYTES_PER_SAMPLE,
                         "samples_per_launch": samples_per_trace_launch},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if gather is not None:
        gather.close()
    for d in dss:
        d.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
