"""bench.py's N>1 path on the device, end to end: two processes (torch.distributed.run,
gloo barriers), each rendering its 8x8 blocks b % 2 == rank with the HIP kernel, and the
gather of rt_shard_pack'ed shards to rank 0 (frame_gather.FrameGather: the IPC pull over
rt_shard_pull_unpack, or the /dev/shm bounce). On a one-GPU box the ranks share the GPU
(bench.py maps LOCAL_RANK onto the GPUs there). Rank 0's gathered frame must be the
one-process frame bit for bit: the md5 of its bytes is compared (position-sensitive: a
swapped block or rank changes it; the f64 frame_sum would not notice). The FrameGather
itself is also driven directly with a different, position-coded frame every step
(tests/gather_worker.py), so both alternating slots are reused and a stale or misplaced
word fails the step it lands in."""
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


def _bench(args, launcher=(), timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([*launcher, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=timeout, cwd=ROOT)
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
    assert two["frame_md5"] == one["frame_md5"]
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
        assert two["frame_md5"] == one["frame_md5"], transport


def test_eight_rank_bench_rehearsal_on_one_gpu():
    """The driver's 8-GPU command shape, rehearsed with 8 processes sharing this box's GPU
    (bench.py maps LOCAL_RANK onto the visible GPUs): 8 gloo ranks, frames in flight on three
    scene handles per rank (--pipeline auto is on for N > 1, RT_FLAG_FRAMES_IN_FLIGHT), 1/8 of
    the C1 frame's blocks per rank, gathered to rank 0 inside the timed region over the IPC pull
    (7 peers, 3 handles each: 24 scenes on one device) and over the /dev/shm bounce. Rank 0's
    frame after warmup 1 + 2 timed steps is the one-process frame bit for bit."""
    common = ["--config", "C1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    one = _bench(common, (sys.executable,))
    for transport in ("ipc", "shm"):
        eight = _bench(["--gpus", "8", "--gather", transport, *common],
                       (sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port())), timeout=420)
        assert eight["n_gpus"] == 8 and eight["scaling"] == "strong"
        assert eight["config"]["gather"] == transport
        assert eight["config"]["pipeline"], "frames in flight are on for N > 1"
        assert eight["frame_md5"] == one["frame_md5"], transport
        assert eight["image_finite"]


@pytest.mark.parametrize("transport,world,lag", [("ipc", 2, False), ("ipc", 3, False), ("shm", 2, False),
                                                 ("ipc", 2, True), ("shm", 2, True), ("ipc", 8, False),
                                                 ("shm", 8, False), ("ipc", 8, True)])
def test_frame_gather_position_coded_frames(transport, world, lag, tmp_path):
    """FrameGather driven directly: 5 steps (both slots reused twice), a ragged 203 x 117
    frame whose every float is distinct and changes each step; rank 0's frame must equal
    it bit for bit after every step (tests/gather_worker.py). `lag`: rank 0's pulls run ~20 ms
    late on its GPU and it never synchronises inside the loop, so the peers run ahead and the
    two-slot reuse rule is what keeps a peer from overwriting a slot still being read."""
    out = tmp_path / "gather.json"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                        os.path.join(ROOT, "tests", "gather_worker.py"), transport, "203", "117", "5", str(out),
                        *(["lag"] if lag else [])],
                       capture_output=True, text=True, env=env, timeout=240 if world < 8 else 420, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["transport"] == transport and res["world"] == world and res["lag"] == lag
    assert len(res["steps"]) == 5
    assert all(st["equal"] for st in res["steps"]), res["steps"]
