"""Data-parallel runtime: one process per GPU, RCCL over xGMI (replaces distributed.py:24-31's
init_process_group("nccl") and the DDP + SyncBatchNorm wrapping of logger.py:54-58).

* `init_dist(local_rank, world_size)` — torch.distributed rendezvous (env://, used only to
  exchange the RCCL unique id) + our own RCCL communicator (libfacevae `fv_comm_*`).
* `DataParallel(module)` — DDP replacement: broadcast of params/buffers from rank 0 once
  (collective C2 of SURVEY.md §2), gradient all-reduce (AVG) in ~25 MB buckets launched
  from post-accumulate-grad hooks on a dedicated comm stream so it overlaps the rest of
  the backward pass (C4); the compute stream waits for the comm stream only at the end.
* SyncBN: BN statistics ([3][C] fp64) and backward sums ([2][C] fp64) are all-reduced on
  the compute stream between the stats and finalize kernels (C5/C6).

`TorchComm` implements the same interface over torch.distributed (gloo) so the bucketing /
averaging / SyncBN plumbing is testable on CPU with world_size 2.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import torch
import torch.distributed as dist

_COMM = None          # installed communicator (RcclComm / TorchComm)
_SYNCBN = True


class RcclComm:
    """fv_comm_* communicator bound to one GPU; collectives are stream-ordered."""

    def __init__(self, rank: int, world_size: int, device: int, uid: bytes):
        from . import _lib as L
        self._L = L
        self.rank, self.world_size, self.device = rank, world_size, device
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        L.call("fv_comm_init", ctypes.addressof(buf), world_size, rank, device, ctypes.byref(h))
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        from . import _lib as L
        buf = (ctypes.c_uint8 * 128)()
        L.call("fv_comm_unique_id", ctypes.addressof(buf))
        return bytes(buf)

    def allreduce_(self, t: torch.Tensor, op: str = "sum", stream=None):
        L = self._L
        s = stream.cuda_stream if stream is not None else L.stream()
        L.call("fv_comm_allreduce", self._h, t.data_ptr(), t.numel(), L.dtype_code(t.dtype),
               1 if op == "avg" else 0, s)
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, stream=None):
        L = self._L
        s = stream.cuda_stream if stream is not None else L.stream()
        L.call("fv_comm_broadcast", self._h, t.data_ptr(), t.numel(), L.dtype_code(t.dtype), root, s)
        return t

    def destroy(self):
        if self._h:
            self._L.call("fv_comm_destroy", self._h)
            self._h = None


class TorchComm:
    """Same interface over torch.distributed (gloo on CPU) — for the CPU tests."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)

    def allreduce_(self, t, op="sum", stream=None):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        if op == "avg":
            t.div_(self.world_size)
        return t

    def broadcast_(self, t, root=0, stream=None):
        dist.broadcast(t, src=root, group=self.group)
        return t

    def destroy(self):
        pass


def install(comm, syncbn: bool = True):
    global _COMM, _SYNCBN
    _COMM, _SYNCBN = comm, syncbn


def get_comm():
    return _COMM


def syncbn_comm():
    if _COMM is not None and _SYNCBN and _COMM.world_size > 1:
        return _COMM
    return None


def get_rank() -> int:
    if _COMM is not None:
        return _COMM.rank
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def get_world_size() -> int:
    if _COMM is not None:
        return _COMM.world_size
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def is_master() -> bool:
    return get_rank() == 0


def init_seeds(seed: int = 1):
    """distributed.py:9-21 (the reference seeds every rank with 1: init_seeds runs before
    init_dist, Appendix A.1)."""
    import random
    import numpy as np
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def init_dist(local_rank: Optional[int] = None, world_size: Optional[int] = None, syncbn: bool = True):
    """Rendezvous via env:// (MASTER_ADDR/PORT, RANK, WORLD_SIZE as torch.distributed.run
    sets them) and create the RCCL communicator of this process's GPU."""
    if local_rank is None:
        local_rank = int(os.environ.get("LOCAL_RANK", 0))
    rank = int(os.environ.get("RANK", local_rank))
    if world_size is None:
        world_size = int(os.environ.get("WORLD_SIZE", 1))
    torch.cuda.set_device(local_rank)
    if world_size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", init_method="env://", world_size=world_size, rank=rank)
    if world_size > 1:
        obj = [RcclComm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = RcclComm(rank, world_size, local_rank, obj[0])
    else:
        comm = None
    install(comm, syncbn)
    return comm


class DataParallel(torch.nn.Module):
    """DistributedDataParallel replacement with bucketed, overlapped gradient all-reduce."""

    def __init__(self, module: torch.nn.Module, comm=None, bucket_cap_mb: float = 25.0):
        super().__init__()
        self.module = module
        self.comm = comm if comm is not None else _COMM
        self.world = self.comm.world_size if self.comm is not None else 1
        params = [p for p in module.parameters() if p.requires_grad]
        self._params = params
        if self.comm is not None and self.world > 1:
            with torch.no_grad():
                for t in list(module.parameters()) + list(module.buffers()):
                    if t.is_floating_point():
                        self.comm.broadcast_(t.data, 0)
        # buckets in reverse registration order (~ the order grads become ready)
        cap = int(bucket_cap_mb * 1024 * 1024 / 4)
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(params):
            if cur and size + p.numel() > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self.buckets.append(cur)
        self._where = {}
        self._flat = []
        for bi, b in enumerate(self.buckets):
            off = 0
            for p in b:
                self._where[id(p)] = (bi, off)
                off += p.numel()
            self._flat.append(None)
            self._flat_n = None
        self._sizes = [sum(p.numel() for p in b) for b in self.buckets]
        self._pending = [0] * len(self.buckets)
        self._cuda = params[0].is_cuda if params else False
        self._comm_stream = torch.cuda.Stream(device=params[0].device) if (self._cuda and self.world > 1) else None
        self._hooks = []
        self._armed = False
        if self.world > 1:
            for p in params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def forward(self, *args, **kwargs):
        self._pending = [len(b) for b in self.buckets]
        self._armed = False
        return self.module(*args, **kwargs)

    def _flat_buf(self, bi, like):
        f = self._flat[bi]
        if f is None or f.device != like.device:
            f = torch.empty(self._sizes[bi], dtype=torch.float32, device=like.device)
            self._flat[bi] = f
        return f

    def _on_grad(self, p):
        bi, off = self._where[id(p)]
        flat = self._flat_buf(bi, p.grad)
        flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
        if not self._armed:
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
            self._armed = True
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi):
        flat = self._flat[bi]
        if self._comm_stream is not None:
            cur = torch.cuda.current_stream(flat.device)
            self._comm_stream.wait_stream(cur)
            with torch.cuda.stream(self._comm_stream):
                self.comm.allreduce_(flat, op="avg", stream=self._comm_stream)
                flat.record_stream(self._comm_stream)
        else:
            self.comm.allreduce_(flat, op="avg")

    def _finish(self):
        for bi, n in enumerate(self._pending):     # params that got no grad this step
            if n != 0 and n != len(self.buckets[bi]):
                raise RuntimeError("DataParallel: a bucket was only partially reduced "
                                   "(unused parameters are not supported)")
        if self._comm_stream is not None:
            torch.cuda.current_stream(self._comm_stream.device).wait_stream(self._comm_stream)
        for bi, b in enumerate(self.buckets):
            if self._pending[bi] != 0:
                continue
            flat = self._flat[bi]
            for p in b:
                _, off = self._where[id(p)]
                p.grad = flat[off:off + p.numel()].view_as(p)
        self._armed = False

    def sync_buffers(self):
        """Broadcast BN running stats / SN u, v from rank 0 (the reference's per-forward C3
        broadcast; identical under SyncBN, so done on demand, e.g. once per epoch)."""
        if self.comm is None or self.world == 1:
            return
        with torch.no_grad():
            for t in self.module.buffers():
                if t.is_floating_point():
                    self.comm.broadcast_(t.data, 0)
