"""Frame assembly for one process per GPU.

The reference renders its tiles on a rayon pool and composites them into one
image (src/renderer.rs:63-95). Here every rank is a process with its own GPU:
rank r renders the 8x8 blocks b with b % n == r (rt_render_params.shard_index /
shard_count) into a full-frame device image, and the frame is gathered to rank 0
without any collective on the data path:

1. rank r packs its blocks into a dense device buffer (rt_shard_pack) and copies
   it with one hipMemcpyAsync D2H into its slot of a POSIX shared-memory buffer
   (/dev/shm, page-locked with hipHostRegister when the runtime allows it);
   rank 0 packs its own blocks straight into its gather buffer on the device;
2. one gloo barrier (the only synchronisation: "every shard has landed");
3. rank 0 copies the other ranks' slots (one contiguous range) H2D and scatters
   all shards into the final image (rt_shard_unpack).

Pure copies, so the assembled frame is the one-device frame bit for bit.
"""
from __future__ import annotations

import mmap
import os
import uuid
from typing import Callable, Optional

import numpy as np

from . import shard_floats, shard_offset, shard_pack, shard_unpack


class FrameGather:
    """Gathers the block-interleaved shards of a W x H frame from `world` ranks to rank 0.

    `pack(d_image, w, h, rank, n, d_packed, stream)` / `unpack(d_all, w, h, n, d_image, stream)`
    default to the HIP kernels (rt_shard_pack / rt_shard_unpack); `device` is the torch
    device of this rank's buffers. Collective calls go to `group` (a gloo group)."""

    def __init__(self, width: int, height: int, rank: int, world: int, device, group=None,
                 pack: Optional[Callable] = None, unpack: Optional[Callable] = None):
        import torch
        import torch.distributed as dist
        self.w, self.h, self.rank, self.world = width, height, rank, world
        self.device = torch.device(device)
        self.group = group
        self._pack = pack or shard_pack
        self._unpack = unpack or shard_unpack
        self.total = shard_offset(width, height, world, world)
        self.off = shard_offset(width, height, rank, world)
        self.cnt = shard_floats(width, height, rank, world)
        self.off1 = shard_offset(width, height, 1, world) if world > 1 else self.total
        # the shared host buffer: created by rank 0, its name broadcast over the gloo group
        name = [f"/dev/shm/rt_gather_{uuid.uuid4().hex}" if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(name, src=0, group=group)
        self.path = name[0]
        nbytes = max(self.total * 4, 4)
        if rank == 0:
            with open(self.path, "wb") as f:
                f.truncate(nbytes)
        if world > 1:
            dist.barrier(group=group)
        self._fd = os.open(self.path, os.O_RDWR)
        self._map = mmap.mmap(self._fd, nbytes)
        self.host = torch.from_numpy(np.frombuffer(self._map, dtype=np.float32, count=max(self.total, 1)))
        self.pinned = False
        if self.device.type == "cuda":
            try:  # page-lock the shared pages so the D2H / H2D copies are true DMA (hipHostRegister)
                rc = torch.cuda.cudart().cudaHostRegister(self.host.data_ptr(), nbytes, 0)
                self.pinned = int(rc) == 0
            except Exception:
                self.pinned = False
        if rank == 0:
            self.d_all = torch.empty(self.total, dtype=torch.float32, device=self.device)
            self.image = torch.zeros(width * height * 3, dtype=torch.float32, device=self.device)
        else:
            self.d_pack = torch.empty(max(self.cnt, 1), dtype=torch.float32, device=self.device)

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
        import torch.distributed as dist
        st = self._stream()
        if self.rank == 0:
            if self.world == 1:
                return d_image
            self._pack(d_image, self.w, self.h, 0, self.world, self.d_all[: self.off1], st)
        else:
            if self.cnt:
                self._pack(d_image, self.w, self.h, self.rank, self.world, self.d_pack[: self.cnt], st)
                self.host[self.off: self.off + self.cnt].copy_(self.d_pack[: self.cnt], non_blocking=self.pinned)
            self._sync()
        dist.barrier(group=self.group)  # every rank's shard is in the shared buffer
        if self.rank == 0:
            if self.total > self.off1:
                self.d_all[self.off1:].copy_(self.host[self.off1: self.total], non_blocking=self.pinned)
            self._unpack(self.d_all, self.w, self.h, self.world, self.image, st)
            return self.image
        return None

    def close(self):
        import torch
        if getattr(self, "_map", None) is None:
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
