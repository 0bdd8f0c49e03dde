"""One rank of the position-sensitive FrameGather check (run by tests/test_gpu_multiprocess.py
under torch.distributed.run; gloo barriers, the HIP gather kernels on the device).

    gather_worker.py TRANSPORT WIDTH HEIGHT STEPS OUT_JSON [lag]

Step k's true frame is distinct at every float (value = index + k / 4, exact in f32 for the
sizes used), so a block written to the wrong place, a slot read one step late, or a stale
peer word changes the assembled frame. Every rank holds that frame on its own blocks and
a rank- and step-dependent negative value everywhere else, so taking a block from a rank
that does not own it is caught too. Rank 0 compares its assembled frame with the true one
bit for bit after every step and writes the per-step verdicts to OUT_JSON.

`lag`: rank 0 never synchronises inside the loop. Before each gather it enqueues a ~20 ms
device sleep, so its pull of step k runs late on the GPU while the peers are already packing
step k+1 (and would pack step k+2 into the slot step k is read from, were the protocol wrong);
it keeps a device copy of each assembled frame, enqueued behind the pull, and compares them all
at the end.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def verdict(got, want):
    bad = (got != want).nonzero()
    return {"equal": bool(bad.numel() == 0), "mismatches": int(bad.numel()),
            "first": int(bad[0].item()) if bad.numel() else None}


def main() -> int:
    transport, w, h, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    lag = len(sys.argv) > 6 and sys.argv[6] == "lag"
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
    verdicts, kept = [], []
    for k in range(steps):
        want = base + 0.25 * k
        img = torch.where(mine, want, torch.full_like(want, -1.0 - rank - 0.125 * k))
        if lag and rank == 0:
            torch.cuda._sleep(40_000_000)  # ~20 ms of device time ahead of this step's pull
        got = g.gather(img)
        if rank == 0:
            if lag:
                kept.append(got.clone())  # in stream order, behind the pull
            else:
                torch.cuda.synchronize()
                kept.append(got)
            if not lag:
                verdicts.append(verdict(kept.pop(), want))
    if rank == 0 and lag:
        torch.cuda.synchronize()
        verdicts = [verdict(f, base + 0.25 * k) for k, f in enumerate(kept)]
    used = g.transport
    g.close()
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"transport": used, "world": world, "lag": lag, "steps": verdicts}, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
