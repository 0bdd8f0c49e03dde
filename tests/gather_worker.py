"""One rank of the position-sensitive FrameGather check (run by tests/test_gpu_multiprocess.py
under torch.distributed.run; gloo barriers, the HIP gather kernels on the device).

    gather_worker.py TRANSPORT WIDTH HEIGHT STEPS OUT_JSON

Step k's true frame is distinct at every float (value = index + k / 4, exact in f32 for the
sizes used), so a block written to the wrong place, a slot read one step late, or a stale
peer word changes the assembled frame. Every rank holds that frame on its own blocks and
a rank- and step-dependent negative value everywhere else, so taking a block from a rank
that does not own it is caught too. Rank 0 compares its assembled frame with the true one
bit for bit after every step and writes the per-step verdicts to OUT_JSON.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    transport, w, h, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import raytracinginoneweekendinrust_amd as rt
    from raytracinginoneweekendinrust_amd.frame_gather import FrameGather

    g = FrameGather(w, h, rank, world, device=f"cuda:{dev}", transport=transport)
    mine = rt.shard_mask(w, h, rank, world, device=f"cuda:{dev}").repeat_interleave(3)
    base = torch.arange(w * h * 3, dtype=torch.float32, device=f"cuda:{dev}")
    verdicts = []
    for k in range(steps):
        want = base + 0.25 * k
        img = torch.where(mine, want, torch.full_like(want, -1.0 - rank - 0.125 * k))
        got = g.gather(img)
        if rank == 0:
            torch.cuda.synchronize()
            bad = (got != want).nonzero()
            verdicts.append({"equal": bool(bad.numel() == 0), "mismatches": int(bad.numel()),
                             "first": int(bad[0].item()) if bad.numel() else None})
    used = g.transport
    g.close()
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"transport": used, "world": world, "steps": verdicts}, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
