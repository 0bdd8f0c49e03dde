"""The N>1 decomposition of bench.py, run with world_size-2 `gloo` ranks on CPU.

Each rank computes its share with bench.rank_work() exactly as on the GPU box,
renders it (the CPU oracle stands in for the device here — the GPU path's own
shard/sample-range semantics are checked bit-exactly in test_gpu_parity.py),
and the shares are exchanged with gloo collectives:
  strong: the composed frame equals the single-process frame bit for bit;
  weak:   the mean of the rank frames equals one render with N*spp samples up to
          float reassociation of the per-pixel sum (rtol 1e-6).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, scaling, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle_ffi as orc
        import raytracinginoneweekendinrust_amd as rt
        cfg = rt.CONFIGS["C3"].scaled(40, 3)
        scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
        params, pixels = bench.rank_work(rt, cfg, rank, world, scaling)
        img = np.zeros((cfg.height, cfg.width, 3), dtype=np.float32)
        _, cnt = orc.render(scene, cfg.camera(), params, out=img, threads=2)
        assert cnt["samples"] == pixels * cfg.spp
        t = torch.from_numpy(img)
        gathered = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        wall = torch.tensor([cnt["seconds"]], dtype=torch.float64)
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((np.stack([g.numpy() for g in gathered]), float(wall.item())))
    finally:
        dist.destroy_process_group()


def run(scaling, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scaling, q)) for r in range(world)]
    for p in procs:
        p.start()
    frames, wall = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return frames, wall


def reference(rt, orc, spp_mult=1):
    cfg = rt.CONFIGS["C3"].scaled(40, 3 * spp_mult)
    scene = rt.Scene.generate(cfg.scene, cfg.scene_seed)
    p = rt.render_params(cfg.width, cfg.height, cfg.spp, cfg.depth, background=cfg.background(), seed=cfg.render_seed)
    img, _ = orc.render(scene, cfg.camera(), p)
    return img


def test_strong_scaling_shards_compose(rt, orc):
    frames, wall = run("strong")
    composed = frames.sum(axis=0)  # disjoint blocks; untouched pixels are 0
    np.testing.assert_array_equal(composed, reference(rt, orc))
    assert wall > 0


def test_weak_scaling_sample_ranges_form_a_progressive_render(rt, orc):
    frames, _ = run("weak")
    assert not np.array_equal(frames[0], frames[1])  # disjoint sample ranges
    np.testing.assert_allclose(frames.mean(axis=0), reference(rt, orc, spp_mult=2), rtol=1e-6, atol=1e-7)
