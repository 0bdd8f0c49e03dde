"""bench.py's N>1 path on the device, end to end: two processes (torch.distributed.run,
gloo barriers), each rendering its 8x8 blocks b % 2 == rank with the HIP kernel, and the
shared-memory gather of rt_shard_pack'ed shards to rank 0 (frame_gather.FrameGather).
On a one-GPU box both ranks share the GPU (bench.py maps LOCAL_RANK onto the GPUs there).
Rank 0's gathered frame must be the one-process frame bit for bit: its frame_sum (the f64
sum of every float of the image) is compared exactly, and both lines must cover the same
W*H*spp samples."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(args, launcher=()):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([*launcher, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_two_rank_bench_gathers_the_one_gpu_frame():
    common = ["--config", "C1", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
    one = _bench(common, (sys.executable,))
    two = _bench(["--gpus", "2", *common],
                 (sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                  "--master-addr", "127.0.0.1", "--master-port", str(_port())))
    assert two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert two["frame_sum"] == one["frame_sum"]
    assert two["image_finite"] and one["image_finite"]
    assert two["rays_per_s"] > 0
    assert two["config"]["gather"] in ("ipc", "shm")


def test_two_rank_bench_back_to_back_frames_over_both_transports():
    """Three frames through the gather's alternating slots (warmup 1 + 2 timed steps) over
    the peer (IPC) transport and over the /dev/shm bounce: rank 0 ends with the one-GPU
    frame bit for bit either way."""
    common = ["--config", "C1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    one = _bench(common, (sys.executable,))
    for transport in ("ipc", "shm"):
        two = _bench(["--gpus", "2", "--gather", transport, *common],
                     (sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                      "--master-addr", "127.0.0.1", "--master-port", str(_port())))
        assert two["config"]["gather"] == transport
        assert two["frame_sum"] == one["frame_sum"], transport
