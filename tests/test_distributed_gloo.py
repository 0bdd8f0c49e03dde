"""The N>1 decomposition of bench.py, run with world_size-2/3 `gloo` ranks on CPU.

Each rank computes its share with bench.rank_work() exactly as on the GPU box and
renders it (the CPU oracle stands in for the device here — the GPU path's own
shard/sample-range semantics are checked bit-exactly in test_gpu_parity.py):
  strong (bench's default): the shards go through the SAME FrameGather the bench
          runs (its shared-memory transport: alternating slots at rt_shard_offset, the
          gloo barrier, rank 0's assembly; three frames back to back), with torch
          restatements of rt_shard_pack / rt_shard_unpack in place of the HIP kernels
          (tested on the device in test_gpu_boundary.py);
          rank 0's frame equals the single-process frame bit for bit;
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


def cpu_pack(img, w, h, r, n, packed, stream=0):
    """Torch restatement of rt_shard_pack: blocks b = r, r+n, ... in order, 64 slots each."""
    bx, nb = (w + 7) // 8, ((w + 7) // 8) * ((h + 7) // 8)
    im = img.view(h, w, 3)
    for k, b in enumerate(range(r, nb, n)):
        x0, y0 = (b % bx) * 8, (b // bx) * 8
        for p in range(64):
            x, y = x0 + (p & 7), y0 + (p >> 3)
            if x < w and y < h:
                packed[(k * 64 + p) * 3: (k * 64 + p) * 3 + 3] = im[y, x]


def cpu_unpack(packed_all, w, h, n, img, stream=0):
    """Torch restatement of rt_shard_unpack: block b from shard b % n, slot b // n."""
    import raytracinginoneweekendinrust_amd as rt
    bx, nb = (w + 7) // 8, ((w + 7) // 8) * ((h + 7) // 8)
    im = img.view(h, w, 3)
    for b in range(nb):
        base = rt.shard_offset(w, h, b % n, n) // 3 + (b // n) * 64
        x0, y0 = (b % bx) * 8, (b // bx) * 8
        for p in range(64):
            x, y = x0 + (p & 7), y0 + (p >> 3)
            if x < w and y < h:
                im[y, x] = packed_all[(base + p) * 3: (base + p) * 3 + 3]


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
        img = np.full((cfg.height, cfg.width, 3), -1.0, dtype=np.float32)  # other ranks' pixels: garbage
        _, cnt = orc.render(scene, cfg.camera(), params, out=img, threads=2)
        assert cnt["samples"] == pixels * cfg.spp
        if scaling == "strong":  # the bench's gather path
            from raytracinginoneweekendinrust_amd.frame_gather import FrameGather
            g = FrameGather(cfg.width, cfg.height, rank, world, "cpu", pack=cpu_pack, unpack=cpu_unpack)
            try:
                assert g.transport == "shm"
                # three frames back to back through the alternating slots: the frame, its
                # double, the frame again (a step must never read another's shards)
                outs = []
                for scale in (1.0, 2.0, 1.0):
                    full = g.gather(torch.from_numpy(img * np.float32(scale)).reshape(-1))
                    if rank == 0:
                        outs.append(full.numpy().reshape(1, cfg.height, cfg.width, 3).copy())
                    else:
                        assert full is None
                if rank == 0:
                    np.testing.assert_array_equal(outs[1], outs[0] * np.float32(2.0))
                    np.testing.assert_array_equal(outs[2], outs[0])
                    q.put((outs[0], cnt["seconds"]))
            finally:
                g.close()
            return
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


@pytest.mark.parametrize("world", [2, 3, 8])
def test_strong_scaling_gather_assembles_the_frame(rt, orc, world):
    # world 8: the bench's 8-GPU decomposition (20 blocks over 8 ranks: 3, 3, 3, 3, 2, 2, 2, 2)
    frames, wall = run("strong", world)
    np.testing.assert_array_equal(frames[0], reference(rt, orc))
    assert wall > 0


def test_weak_scaling_sample_ranges_form_a_progressive_render(rt, orc):
    frames, _ = run("weak")
    assert not np.array_equal(frames[0], frames[1])  # disjoint sample ranges
    np.testing.assert_allclose(frames.mean(axis=0), reference(rt, orc, spp_mult=2), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("w,h,n", [(203, 117, 2), (1200, 800, 8), (9, 1, 3), (64, 64, 64)])
def test_ipc_probe_block_ranks_follow_the_shard_map(rt, w, h, n):
    # FrameGather's IPC probe expects every pulled pixel to hold its rank's value: the rank map it
    # compares against is the same 8x8-block interleave as rt.shard_mask / rt_shard_pack
    from raytracinginoneweekendinrust_amd.frame_gather import MAX_PULL_RANKS, block_ranks
    ranks = block_ranks(w, h, n).reshape(-1)
    for r in range(n):
        np.testing.assert_array_equal(ranks == r, rt.shard_mask(w, h, r, n).numpy())
    assert MAX_PULL_RANKS == 64
