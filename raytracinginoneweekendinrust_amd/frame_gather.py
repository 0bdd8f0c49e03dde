"""Frame assembly for one process per GPU.

The reference renders its tiles on a rayon pool and composites them into one
image (src/renderer.rs:63-95). Here every rank is a process with its own GPU:
rank r renders the 8x8 blocks b with b % n == r (rt_render_params.shard_index /
shard_count) into a full-frame device image, and the frame is gathered to rank 0
without any collective on the data path:

1. rank r packs its blocks into a dense device buffer (rt_shard_pack); rank 0
   packs its own blocks straight into its gather buffer on the device;
2. transport, one of
   * "ipc" (default on GPUs): rank 0's gather buffer is exported once with
     hipIpcGetMemHandle (rt_ipc_export) and mapped by every other rank
     (rt_ipc_open); a rank copies its packed shard straight into its slot with one
     device-to-device hipMemcpyAsync (rt_copy_async) — over xGMI between GPUs, the
     north-star's "hipMemcpyAsync gather to rank 0", one hop;
   * "shm" (fallback, and the CPU tests): one hipMemcpyAsync D2H into the rank's
     slot of a POSIX shared-memory buffer (/dev/shm, page-locked with
     hipHostRegister when the runtime allows it), then rank 0 copies the other
     ranks' slots H2D;
3. one gloo barrier ("every shard has landed"); rank 0 scatters all shards into
   the final image (rt_shard_unpack).

The gather buffer has two slots used in alternate steps, and rank 0 waits for its
previous unpack before it enters a step's barrier: a rank writes slot s of step k+2
only after the barrier of step k+1, by when rank 0's unpack of step k (the last
reader of slot s) has completed, so a fast rank can never overwrite a shard rank 0
is still reading. Pure copies, so the assembled frame is the
one-device frame bit for bit.
"""
from __future__ import annotations

import mmap
import os
import uuid
from typing import Callable, Optional

import numpy as np

from . import shard_floats, shard_offset, shard_pack, shard_unpack

SLOTS = 2  # gather-buffer slots, used in alternate steps


class FrameGather:
    """Gathers the block-interleaved shards of a W x H frame from `world` ranks to rank 0.

    `pack(d_image, w, h, rank, n, d_packed, stream)` / `unpack(d_all, w, h, n, d_image, stream)`
    default to the HIP kernels (rt_shard_pack / rt_shard_unpack); `device` is the torch
    device of this rank's buffers. Collective calls go to `group` (a gloo group).
    `transport`: "auto" (ipc on GPUs when every rank can map rank 0's buffer, else shm),
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
        self._peer = None      # ranks > 0, ipc: rank 0's gather buffer mapped here
        self.host = None
        self.pinned = False
        cuda = self.device.type == "cuda"
        if rank == 0:
            self.d_all = torch.empty(SLOTS * max(self.total, 1), dtype=torch.float32, device=self.device)
            self.image = torch.zeros(width * height * 3, dtype=torch.float32, device=self.device)
        else:
            self.d_pack = torch.empty(max(self.cnt, 1), dtype=torch.float32, device=self.device)
        self.transport = "shm"
        if world > 1 and cuda and transport in ("auto", "ipc"):
            self.transport = self._open_ipc(transport == "ipc")
        if world > 1 and self.transport == "shm":
            self._open_shm()

    # --- transports ------------------------------------------------------------
    def _open_ipc(self, required: bool) -> str:
        """Rank 0 exports its gather buffer, the others map it; every rank must succeed
        (a MIN over the gloo group), else all fall back to shm together."""
        import torch
        import torch.distributed as dist
        from . import ipc_export, ipc_open
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        handle = [None]
        ok = 1
        if self.rank == 0:
            try:
                handle[0] = ipc_export(self.d_all.data_ptr(), dev)
            except Exception:
                ok = 0
        dist.broadcast_object_list(handle, src=0, group=self.group)
        if self.rank != 0 and handle[0] is not None:
            try:
                self._peer = ipc_open(handle[0], dev)
                if self.cnt:  # one real peer copy into this rank's slot, so a transport that maps but
                    from . import copy_async  # cannot copy falls back here, not inside a timed step
                    copy_async(self._peer + self.off * 4, self.d_pack.data_ptr(), 4, self._stream())
                    self._sync()
            except Exception:
                ok = 0
        elif handle[0] is None:
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 1:
            return "ipc"
        if self._peer is not None:
            self._close_ipc()
        if required:
            raise RuntimeError("FrameGather: IPC transport unavailable on some rank")
        return "shm"

    def _close_ipc(self):
        import torch
        from . import ipc_close
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        try:
            ipc_close(self._peer, dev)
        except Exception:
            pass
        self._peer = None

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
        base = (self.step % SLOTS) * self.total
        self.step += 1
        if self.rank == 0:
            self._pack(d_image, self.w, self.h, 0, self.world, self.d_all[base: base + self.off1], st)
            if self._unpacked is not None:  # the unpack of the previous step (last reader of the other slot)
                self._unpacked.synchronize()
        else:
            if self.cnt:
                self._pack(d_image, self.w, self.h, self.rank, self.world, self.d_pack[: self.cnt], st)
                if self.transport == "ipc":
                    from . import copy_async
                    copy_async(self._peer + (base + self.off) * 4, self.d_pack.data_ptr(), self.cnt * 4, st)
                else:
                    self.host[base + self.off: base + self.off + self.cnt].copy_(self.d_pack[: self.cnt],
                                                                                 non_blocking=self.pinned)
            self._sync()
        dist.barrier(group=self.group)  # every rank's shard is in rank 0's slot
        if self.rank != 0:
            return None
        if self.transport == "shm" and self.total > self.off1:
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
        if self._peer is not None:
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
