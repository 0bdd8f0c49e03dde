"""Frame assembly for one process per GPU.

The reference renders its tiles on a rayon pool and composites them into one
image (src/renderer.rs:63-95). Here every rank is a process with its own GPU:
rank r of n renders the 8x8 blocks b with b % n == r (rt_render_params.shard_index /
shard_count) into a full-frame device image, and the frame is assembled on rank 0
without any collective on the data path:

1. every rank r > 0 packs its blocks into a dense device buffer (rt_shard_pack,
   whose threads end with a system-scope release) and synchronises its stream;
2. one gloo barrier ("every shard is packed");
3. transport, one of
   * "ipc" (default on GPUs), a PULL over xGMI: every rank r > 0 exported its
     two-slot packed-shard buffer once (rt_ipc_export) and rank 0 mapped them all
     (rt_ipc_open); rank 0 starts from its own rendered image (its blocks) and one
     kernel, rt_shard_pull_unpack, reads every other rank's blocks straight out of
     the peers' memory (system-scope acquire fence, then system-scope loads) into
     it — one hop, no intermediate copy, and the visibility of the peers' words
     rests on the LLVM AMDGPU memory model (release by the writer's threads, host
     barrier, acquire by the reader's), not on a dispatch default;
   * "shm" (fallback, and the CPU tests): one hipMemcpyAsync D2H of the packed shard
     into the rank's slot of a POSIX shared-memory buffer (/dev/shm, page-locked
     with hipHostRegister when the runtime allows it, rank 0 packing its own shard
     into the same layout), then rank 0 copies the other slots H2D and scatters all
     shards (rt_shard_unpack).

Slots alternate between steps, and rank 0 waits for its previous step's assembly
before it enters a step's barrier: a rank writes slot s of step k+2 only after the
barrier of step k+1, by when rank 0's read of step k (the last reader of slot s)
has completed, so a fast rank can never overwrite a shard rank 0 is still reading
(ADVICE r02). Pure copies, so the assembled frame is the one-device frame bit for
bit (tests/test_gpu_multiprocess.py compares whole frames, step by step).
"""
from __future__ import annotations

import mmap
import os
import uuid
from typing import Callable, Optional

import numpy as np

from . import shard_floats, shard_offset, shard_pack, shard_unpack

SLOTS = 2  # gather-buffer slots, used in alternate steps
MAX_PULL_RANKS = 64  # rt_shard_pull_unpack's peer table (gather.hip kMaxPullRanks)


def block_ranks(width: int, height: int, world: int) -> np.ndarray:
    """The rank that renders each pixel (row-major H*W): 8x8 block b goes to rank b % world."""
    bx = (width + 7) // 8
    y, x = np.mgrid[0:height, 0:width]
    return ((y // 8) * bx + x // 8) % world


class FrameGather:
    """Gathers the block-interleaved shards of a W x H frame from `world` ranks to rank 0.

    `pack(d_image, w, h, rank, n, d_packed, stream)` / `unpack(d_all, w, h, n, d_image, stream)`
    default to the HIP kernels (rt_shard_pack / rt_shard_unpack); `device` is the torch
    device of this rank's buffers. Collective calls go to `group` (a gloo group).
    `transport`: "auto" (ipc on GPUs when rank 0 can map and read every rank's buffer, else shm),
    "ipc" or "shm"; the one in use is `self.transport`."""

    def __init__(self, width: int, height: int, rank: int, world: int, device, group=None,
                 pack: Optional[Callable] = None, unpack: Optional[Callable] = None, transport: str = "auto"):
        import torch
        import torch.distributed as dist
        if transport not in ("auto", "ipc", "shm"):
            raise ValueError(f"transport {transport!r}")
        self.w, self.h, self.rank, self.world = width, height, rank, world
        self.device = torch.device(device)
        self.group = group
        self._pack = pack or shard_pack
        self._unpack = unpack or shard_unpack
        self.total = shard_offset(width, height, world, world)
        self.off = shard_offset(width, height, rank, world)
        self.cnt = shard_floats(width, height, rank, world)
        self.off1 = shard_offset(width, height, 1, world) if world > 1 else self.total
        self.step = 0
        self._unpacked = None  # rank 0: event recorded after the last unpack
        self._map = None
        self.host = None
        self.pinned = False
        cuda = self.device.type == "cuda"
        self._peers = []       # rank 0, ipc: every rank's mapped two-slot packed buffer (entry 0 unused)
        self._peer_cnt = []    # rank 0, ipc: floats per slot of each rank's buffer
        if rank == 0:
            self.image = torch.zeros(width * height * 3, dtype=torch.float32, device=self.device)
        else:  # two slots of this rank's packed shard (alternate steps)
            self.d_pack = torch.empty(SLOTS * max(self.cnt, 1), dtype=torch.float32, device=self.device)
        self.transport = "shm"
        if world > 1 and cuda and transport in ("auto", "ipc"):
            self.transport = self._open_ipc(transport == "ipc")
        if world > 1 and self.transport == "shm":
            if rank == 0:
                self.d_all = torch.empty(SLOTS * max(self.total, 1), dtype=torch.float32, device=self.device)
            self._open_shm()

    # --- transports ------------------------------------------------------------
    def _open_ipc(self, required: bool) -> str:
        """Every rank r > 0 fills slot 0 of its packed buffer with r + 0.5 and exports it; rank 0
        maps them all and pulls a whole probe frame through them with rt_shard_pull_unpack, the
        kernel every gather runs (system-scope acquire and loads), checking that each block holds
        its rank's value: a mapping that the kernel's loads cannot read, or that delivers nothing
        or stale data, is caught here. The pull kernel takes at most 64 ranks. Every rank must
        succeed (a MIN over the gloo group), else all fall back to shm together."""
        import torch
        import torch.distributed as dist
        from . import ipc_export, ipc_open, shard_pull_unpack
        dev = self._dev()
        ok = 1 if self.world <= MAX_PULL_RANKS else 0
        handle = None
        if self.rank != 0 and ok:
            try:
                self.d_pack[: max(self.cnt, 1)].fill_(self.rank + 0.5)
                self._sync()
                handle = ipc_export(self.d_pack.data_ptr(), dev)
            except Exception:
                ok = 0
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=self.group)
        if self.rank == 0 and ok:
            self._peers, self._peer_cnt = [0], [0]
            try:
                for r in range(1, self.world):
                    cnt = shard_floats(self.w, self.h, r, self.world)
                    if handles[r] is None:
                        raise RuntimeError(f"rank {r} exported no buffer")
                    self._peers.append(ipc_open(handles[r], dev))
                    self._peer_cnt.append(max(cnt, 1))
                probe = torch.full((self.w * self.h * 3,), -1.0, dtype=torch.float32, device=self.device)
                shard_pull_unpack(self._peers, self.w, self.h, probe, self._stream())
                self._sync()
                want = torch.from_numpy(block_ranks(self.w, self.h, self.world).astype(np.float32) + 0.5)
                want[want == 0.5] = -1.0  # rank 0's blocks are not pulled
                got = probe.view(self.h * self.w, 3).cpu()
                if not torch.equal(got, want.view(-1, 1).expand(-1, 3)):
                    raise RuntimeError("IPC probe frame differs from the ranks' values")
            except Exception:
                ok = 0
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 1:
            return "ipc"
        self._close_ipc()
        if required:
            raise RuntimeError("FrameGather: IPC transport unavailable on some rank")
        return "shm"

    def _dev(self) -> int:
        import torch
        return self.device.index if self.device.index is not None else torch.cuda.current_device()

    def _close_ipc(self):
        from . import ipc_close
        for ptr in self._peers[1:]:
            try:
                ipc_close(ptr, self._dev())
            except Exception:
                pass
        self._peers, self._peer_cnt = [], []

    def _open_shm(self):
        import torch
        import torch.distributed as dist
        # the shared host buffer: created by rank 0, its name broadcast over the gloo group
        name = [f"/dev/shm/rt_gather_{uuid.uuid4().hex}" if self.rank == 0 else None]
        dist.broadcast_object_list(name, src=0, group=self.group)
        self.path = name[0]
        nbytes = max(SLOTS * self.total * 4, 4)
        if self.rank == 0:
            with open(self.path, "wb") as f:
                f.truncate(nbytes)
        dist.barrier(group=self.group)
        self._fd = os.open(self.path, os.O_RDWR)
        self._map = mmap.mmap(self._fd, nbytes)
        self.host = torch.from_numpy(np.frombuffer(self._map, dtype=np.float32, count=max(SLOTS * self.total, 1)))
        if self.device.type == "cuda":
            try:  # page-lock the shared pages so the D2H / H2D copies are true DMA (hipHostRegister)
                rc = torch.cuda.cudart().cudaHostRegister(self.host.data_ptr(), nbytes, 0)
                self.pinned = int(rc) == 0
            except Exception:
                self.pinned = False

    # --- the gather ------------------------------------------------------------
    def _stream(self):
        import torch
        return torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0

    def _sync(self):
        import torch
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    def gather(self, d_image):
        """This rank's shard of `d_image` (W*H*3 float32 on self.device, the rank's blocks
        rendered) to rank 0; returns rank 0's assembled image tensor, None elsewhere.
        Work is issued on torch's current stream (where the render was launched)."""
        import torch
        import torch.distributed as dist
        st = self._stream()
        if self.world == 1:
            return d_image if self.rank == 0 else None
        slot = self.step % SLOTS
        self.step += 1
        if self.rank == 0:
            if self._unpacked is not None:  # the previous step's assembly (last reader of the other slot)
                self._unpacked.synchronize()
            if self.transport == "ipc":
                self.image.copy_(d_image)  # rank 0's own blocks; the others are pulled below
            else:
                base = slot * self.total
                self._pack(d_image, self.w, self.h, 0, self.world, self.d_all[base: base + self.off1], st)
        elif self.cnt:
            packed = self.d_pack[slot * self.cnt: (slot + 1) * self.cnt]
            self._pack(d_image, self.w, self.h, self.rank, self.world, packed, st)
            if self.transport == "shm":
                base = slot * self.total
                self.host[base + self.off: base + self.off + self.cnt].copy_(packed, non_blocking=self.pinned)
        if self.rank != 0:
            self._sync()  # the shard is packed (ipc) or in the shared slot (shm)
        dist.barrier(group=self.group)  # every rank's shard is ready for rank 0
        if self.rank != 0:
            return None
        if self.transport == "ipc":
            from . import shard_pull_unpack
            ptrs = [0] + [self._peers[r] + slot * self._peer_cnt[r] * 4 for r in range(1, self.world)]
            shard_pull_unpack(ptrs, self.w, self.h, self.image, st)
        else:
            base = slot * self.total
            if self.total > self.off1:
                self.d_all[base + self.off1: base + self.total].copy_(self.host[base + self.off1: base + self.total],
                                                                      non_blocking=self.pinned)
            self._unpack(self.d_all[base: base + self.total], self.w, self.h, self.world, self.image, st)
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._unpacked = ev
        return self.image

    def close(self):
        import torch
        if self._peers:
            self._close_ipc()
        if self._map is None:
            return
        if self.pinned:
            try:
                torch.cuda.cudart().cudaHostUnregister(self.host.data_ptr())
            except Exception:
                pass
        self.host = None
        try:
            self._map.close()
        except BufferError:
            pass
        os.close(self._fd)
        self._map = None
        if self.rank == 0:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass
