"""Data-parallel runtime: one process per GPU, RCCL over xGMI (replaces distributed.py:9-31's
init_seeds / init_process_group("nccl") and the DDP + SyncBatchNorm wrapping of
logger.py:54-58).

* `init_dist(local_rank, world_size, backend="nccl")` — the reference signature
  (distributed.py:24).  torch.distributed is initialised over env:// with gloo and used only
  for the rendezvous (the RCCL unique id); `backend="nccl"` then creates our own RCCL
  communicator (libfacevae `fv_comm_*`), `backend="gloo"` a TorchComm (CPU tests, or several
  ranks sharing one GPU, which RCCL refuses).
* `comm_from_process_group()` — the same, for a caller that initialised torch.distributed
  itself (e.g. the reference `init_dist`): FaceVAETrainer calls it, so a reference-style
  launch never trains unsynchronised.
* `DataParallel(module)` — DDP replacement: broadcast of params/buffers from rank 0 once
  (collective C2 of SURVEY.md §2), gradient all-reduce (AVG) in buckets launched from
  post-accumulate-grad hooks so it overlaps the rest of the backward pass (C4).  Bucketing
  follows DDP: a small first bucket (1 MB, `_DEFAULT_FIRST_BUCKET_BYTES`) so the first
  all-reduce starts as soon as the last layer's gradients exist, then `bucket_cap_mb` (25)
  buckets; one dtype per bucket; optional bf16 gradient compression (`grad_dtype`).
* SyncBN (C5/C6): BN statistics ([3][C] fp64, row 0 = the per-rank pixel count, so uneven
  shards normalise correctly) and the backward sums ([2][C] fp64) are all-reduced in stream
  order between the statistics and finalize kernels.

Ordering: every RCCL collective of a process is issued on ONE comm stream per communicator
(as torch's ProcessGroupNCCL does), fenced against the compute stream with stream waits, and
every rank issues them in the same host order (the autograd engine walks the same graph on
every rank).  No reliance on cross-stream ordering inside RCCL.

`TorchComm` implements the same interface over torch.distributed (gloo) so the bucketing /
averaging / SyncBN plumbing is testable on CPU with world_size 2.
"""
from __future__ import annotations

import ctypes
import os
import random
import sys
import threading
import time
from collections import deque
from typing import Callable, Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist


_COMM = None          # installed communicator (RcclComm / TorchComm)
_SYNCBN = True
_SEGMENTS = None      # graph.SegmentRecorder while a multi-process step is being captured


def _deferred(op):
    """Inside a segmented capture (graph.StepGraph at world > 1) a collective is not issued: it
    ends the current graph segment and is recorded as `op`, which the replay runs eagerly
    between the segments.  Returns True when the call was deferred."""
    if _SEGMENTS is None:
        return False
    _SEGMENTS.cut(op)
    return True

FIRST_BUCKET_MB = 1.0   # torch/nn/parallel/distributed.py _DEFAULT_FIRST_BUCKET_BYTES

# failure detection: a collective still pending after COMM_TIMEOUT_S seconds, or an RCCL async
# error, ends the process (see CommWatchdog)
COMM_TIMEOUT_S = float(os.environ.get("FV_COMM_TIMEOUT", "600"))
COMM_POLL_S = float(os.environ.get("FV_COMM_POLL", "1.0"))

# ncclResult_t values that are not failures
_NCCL_OK, _NCCL_IN_PROGRESS = 0, 7


class CommWatchdog:
    """Fail-fast for the collectives of one communicator (the reference's
    mp.spawn tears every rank down when one raises, train.py:54, and torch's ProcessGroupNCCL
    watchdog aborts a timed-out collective).

    Every issued collective is tracked as (done(), issue time, name).  A daemon thread polls
    every `poll_s` while anything is pending: completed entries are dropped, the communicator's
    asynchronous error is queried (`async_error()` -> ncclResult_t), and an error other than
    success / in-progress, or an entry pending for more than `timeout_s`, calls `abort()` (RCCL
    abandons the outstanding collectives) and then `exit_fn(1)` after printing the reason with
    the rank to stderr.  `exit_fn` is os._exit: the process ends without running atexit
    handlers that could block on the dead communicator, and never re-execs.  While a segmented
    graph capture is in progress (no collective is issued then) the thread does not poll."""

    def __init__(self, rank: int, async_error: Callable[[], int], abort: Callable[[], None],
                 timeout_s: float = COMM_TIMEOUT_S, poll_s: float = COMM_POLL_S,
                 exit_fn: Callable[[int], None] = os._exit):
        self.rank, self._async_error, self._abort = rank, async_error, abort
        self.timeout_s, self.poll_s, self._exit = timeout_s, poll_s, exit_fn
        self._pending = deque()
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.failed: Optional[str] = None
        self._thread = threading.Thread(target=self._run, name=f"fv-comm-watchdog-{rank}", daemon=True)
        self._thread.start()

    def track(self, done: Callable[[], bool], what: str):
        with self._lock:
            self._pending.append((done, time.monotonic(), what))

    def pending(self) -> int:
        with self._lock:
            return len(self._pending)

    def check(self) -> Optional[str]:
        """One poll; returns the failure reason (None while healthy)."""
        with self._lock:
            while self._pending and self._pending[0][0]():
                self._pending.popleft()
            oldest = self._pending[0] if self._pending else None
        if oldest is None:
            return None
        r = self._async_error()
        if r not in (_NCCL_OK, _NCCL_IN_PROGRESS):
            return f"RCCL asynchronous error {r} while {oldest[2]} was pending"
        age = time.monotonic() - oldest[1]
        if age > self.timeout_s:
            return f"{oldest[2]} pending for {age:.0f} s (> FV_COMM_TIMEOUT {self.timeout_s:.0f} s): a peer is dead or stuck"
        return None

    def _fail(self, why: str):
        self.failed = why
        print(f"[facevae rank {self.rank}] communicator failure: {why}; aborting the communicator and exiting",
              file=sys.stderr, flush=True)
        try:
            self._abort()
        finally:
            self._exit(1)

    def _run(self):
        while not self._stop.wait(self.poll_s):
            if _SEGMENTS is not None:
                continue
            try:
                why = self.check()
            except Exception as e:          # a failing query is a failure too
                why = f"watchdog query failed: {e}"
            if why is not None:
                self._fail(why)
                return

    def stop(self):
        self._stop.set()
        self._thread.join(timeout=5 * self.poll_s + 1)


class RcclComm:
    """fv_comm_* communicator bound to one GPU.  All of its collectives run on its own comm
    stream, fenced against the caller's stream (see module docstring)."""

    def __init__(self, rank: int, world_size: int, device: int, uid: bytes):
        from . import _lib as L
        self._L = L
        self.rank, self.world_size, self.device = rank, world_size, device
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        L.call("fv_comm_init", ctypes.addressof(buf), world_size, rank, device, ctypes.byref(h))
        self._h = h
        self.stream = torch.cuda.Stream(device=device)
        self.watchdog = CommWatchdog(rank, self.async_error, self.abort) if world_size > 1 else None

    @staticmethod
    def unique_id() -> bytes:
        from . import _lib as L
        buf = (ctypes.c_uint8 * 128)()
        L.call("fv_comm_unique_id", ctypes.addressof(buf))
        return bytes(buf)

    def async_error(self) -> int:
        """ncclCommGetAsyncError of the communicator (0 = success, 7 = in progress)."""
        r = ctypes.c_int(0)
        self._L.call("fv_comm_async_error", self._h, ctypes.byref(r))
        return r.value

    def count(self) -> int:
        """Ranks the RCCL communicator spans (ncclCommCount)."""
        n = ctypes.c_int(0)
        self._L.call("fv_comm_count", self._h, ctypes.byref(n))
        return n.value

    def abort(self):
        """ncclCommAbort: abandon the outstanding collectives and free the communicator."""
        h, self._h = self._h, None
        if h:
            self._L.query("fv_comm_abort", h)

    def _launch(self, fn, t: torch.Tensor, wait_back: bool, what: str = "collective"):
        if self._h is None:
            raise RuntimeError("RcclComm: the communicator was destroyed or aborted")
        cur = torch.cuda.current_stream(t.device)
        self.stream.wait_stream(cur)
        fn(self.stream.cuda_stream)
        if self.watchdog is not None:
            ev = torch.cuda.Event()
            ev.record(self.stream)
            self.watchdog.track(ev.query, f"{what} of {t.numel()} x {t.dtype}")
        t.record_stream(self.stream)
        if wait_back:
            cur.wait_stream(self.stream)
        return t

    def allreduce_(self, t: torch.Tensor, op: str = "sum", wait_back: bool = True):
        """In-place all-reduce (op "sum" or "avg") on the comm stream; with wait_back the
        caller's stream waits for it (SyncBN), otherwise the caller fences later (buckets)."""
        if _deferred(lambda: self.allreduce_(t, op, wait_back)):
            return t
        L = self._L
        code = {"sum": 0, "avg": 1, "max": 2}[op]
        return self._launch(lambda s: L.call("fv_comm_allreduce", self._h, t.data_ptr(), t.numel(),
                                             L.dtype_code(t.dtype), code, s), t, wait_back, f"all-reduce ({op})")

    def broadcast_(self, t: torch.Tensor, root: int = 0, wait_back: bool = True):
        if _deferred(lambda: self.broadcast_(t, root, wait_back)):
            return t
        L = self._L
        return self._launch(lambda s: L.call("fv_comm_broadcast", self._h, t.data_ptr(), t.numel(),
                                             L.dtype_code(t.dtype), root, s), t, wait_back, "broadcast")

    def fence(self, device=None):
        """Make the caller's stream wait for every collective issued so far."""
        if _deferred(lambda: self.fence(device)):
            return
        torch.cuda.current_stream(device).wait_stream(self.stream)

    def destroy(self):
        if self.watchdog is not None:
            self.watchdog.stop()
            self.watchdog = None
        if self._h:
            self._L.call("fv_comm_destroy", self._h)
            self._h = None


class TorchComm:
    """Same interface over torch.distributed (gloo): synchronous, so no stream fencing."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)

    def allreduce_(self, t, op="sum", wait_back=True):
        if _deferred(lambda: self.allreduce_(t, op, wait_back)):
            return t
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM, group=self.group)
        if op == "avg":
            t.div_(self.world_size)
        return t

    def broadcast_(self, t, root=0, wait_back=True):
        if _deferred(lambda: self.broadcast_(t, root, wait_back)):
            return t
        dist.broadcast(t, src=root, group=self.group)
        return t

    def fence(self, device=None):
        pass

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
    """distributed.py:34-40: torch.distributed's rank (0 when not initialised)."""
    if _COMM is not None:
        return _COMM.rank
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def get_world_size() -> int:
    if _COMM is not None:
        return _COMM.world_size
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def is_master() -> bool:
    return get_rank() == 0


def init_seeds(cuda_deterministic: bool = True):
    """distributed.py:9-21: seed = 1 + rank for python, numpy and torch (CPU and every GPU).
    train.py:12 calls it BEFORE init_dist, so the rank is 0 and every rank seeds 1 (SURVEY.md
    Appendix A.1).  The cuDNN flags have no counterpart here (no cuDNN on this path).  The
    FaceVAE step's HIP kernels are deterministic either way (no float atomics, fixed reduction
    orders), the §8(f)2 warp path included: grid_sample3d's input gradient gathers buckets
    ordered by voxel index (warp.hip gs_bucket_sort)."""
    seed = 1 + get_rank()
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    return seed


def _rccl_from_group(local_rank: int) -> RcclComm:
    rank, world = dist.get_rank(), dist.get_world_size()
    obj = [RcclComm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return RcclComm(rank, world, local_rank, obj[0])


def init_dist(local_rank: Optional[int] = None, world_size: Optional[int] = None, backend: str = "nccl",
              syncbn: bool = True):
    """distributed.py:24-31 with the reference signature.  Rendezvous via env:// (MASTER_ADDR /
    MASTER_PORT; RANK defaults to local_rank as in the reference's mp.spawn launch), then
    `backend` "nccl" -> our RCCL communicator on cuda:local_rank, "gloo" -> TorchComm.  The
    reference also switches on torch.autograd anomaly detection here (distributed.py:26); it
    changes no numerics and is left off."""
    if local_rank is None:
        local_rank = int(os.environ.get("LOCAL_RANK", 0))
    rank = int(os.environ.get("RANK", local_rank))
    if world_size is None:
        world_size = int(os.environ.get("WORLD_SIZE", 1))
    if backend not in ("nccl", "rccl", "gloo"):
        raise ValueError(f"init_dist: backend {backend!r} (nccl/rccl or gloo)")
    if torch.cuda.is_available():
        # gloo: several ranks may share a GPU (RCCL needs one GPU per rank)
        torch.cuda.set_device(local_rank if backend != "gloo" else local_rank % torch.cuda.device_count())
    if world_size > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", init_method="env://", world_size=world_size, rank=rank)
    comm = None
    if world_size > 1:
        comm = TorchComm() if backend == "gloo" else _rccl_from_group(local_rank)
    install(comm, syncbn)
    return comm


def comm_from_process_group(syncbn: bool = True):
    """Communicator for a process whose torch.distributed group was initialised elsewhere
    (e.g. by the reference's init_dist with backend "nccl"): an RCCL communicator on the
    current device for an nccl group, a TorchComm for gloo.  Installed and returned."""
    if not (dist.is_available() and dist.is_initialized()):
        raise RuntimeError("comm_from_process_group: torch.distributed is not initialised")
    if dist.get_world_size() == 1:
        install(None, syncbn)
        return None
    backend = str(dist.get_backend()).lower()
    if backend in ("nccl", "rccl"):
        comm = _rccl_from_group(torch.cuda.current_device())
    elif backend == "gloo":
        comm = TorchComm()
    else:
        raise RuntimeError(f"comm_from_process_group: unsupported torch.distributed backend {backend!r}")
    install(comm, syncbn)
    return comm


def plan_buckets(params, bucket_cap_mb: float = 25.0, first_bucket_mb: float = FIRST_BUCKET_MB):
    """DDP bucket assignment: parameters in reverse registration order (~ the order their
    gradients become ready in backward), one dtype per bucket, the first bucket capped at
    `first_bucket_mb` and the rest at `bucket_cap_mb` (in bytes of the gradient dtype)."""
    buckets: List[List[torch.nn.Parameter]] = []
    cur: Dict[torch.dtype, List] = {}
    size: Dict[torch.dtype, int] = {}

    def cap_bytes():
        return (first_bucket_mb if not buckets else bucket_cap_mb) * 1024 * 1024

    for p in reversed(list(params)):
        dt = p.dtype
        nbytes = p.numel() * p.element_size()
        if cur.get(dt) and size[dt] + nbytes > cap_bytes():
            buckets.append(cur[dt])
            cur[dt], size[dt] = [], 0
        cur.setdefault(dt, []).append(p)
        size[dt] = size.get(dt, 0) + nbytes
    for dt, b in cur.items():
        if b:
            buckets.append(b)
    return buckets


class DataParallel(torch.nn.Module):
    """DistributedDataParallel replacement with bucketed, overlapped gradient all-reduce.

    grad_dtype: None (all-reduce in the parameter dtype, the reference's fp32) or
    torch.bfloat16 (compressed: gradients cast into a bf16 flat buffer, averaged, cast back;
    halves the xGMI bytes, labelled in bench output)."""

    def __init__(self, module: torch.nn.Module, comm=None, bucket_cap_mb: float = 25.0,
                 first_bucket_mb: float = FIRST_BUCKET_MB, grad_dtype: Optional[torch.dtype] = None):
        super().__init__()
        self.module = module
        self.comm = comm if comm is not None else _COMM
        self.world = self.comm.world_size if self.comm is not None else 1
        params = [p for p in module.parameters() if p.requires_grad]
        self._params = params
        self.grad_dtype = grad_dtype
        if self.comm is not None and self.world > 1:
            with torch.no_grad():
                for t in list(module.parameters()) + list(module.buffers()):
                    if t.is_floating_point():
                        self.comm.broadcast_(t.data, 0)
        self.buckets = plan_buckets(params, bucket_cap_mb, first_bucket_mb)
        self._where = {}
        for bi, b in enumerate(self.buckets):
            off = 0
            for p in b:
                self._where[id(p)] = (bi, off)
                off += p.numel()
        self._sizes = [sum(p.numel() for p in b) for b in self.buckets]
        self._flat: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        self._pending = [0] * len(self.buckets)
        self.launch_order: List[int] = []      # bucket indices in launch order, last backward
        self._hooks = []
        self._armed = False
        self._fp8_key = None
        if self.world > 1:
            for p in params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _global_fp8(self, on: bool):
        """fp8 operands (config C5): one scale per operand for the whole global batch, as
        SyncBN's statistics (ops.quantize_fp8_site seeds through the communicator, the convs
        leave their amax in-flight and _sync_fp8 rolls every site once per step).  Scoped to
        this wrapper's training step -- switched on by forward, off by the end-of-backward
        callback -- so an fp8 module used outside it (an eval copy, a second model) rolls its
        own sites and never issues a collective the other ranks do not match."""
        from . import _lib, ops
        ops.FP8_GLOBAL = self.comm if on else None
        _lib.call("fv_fp8_set_deferred_roll", 1 if on else 0)

    def forward(self, *args, **kwargs):
        self._pending = [len(b) for b in self.buckets]
        self._armed = False
        self.launch_order = []
        if self.world > 1:
            self._global_fp8(self.module.training and torch.is_grad_enabled())
        return self.module(*args, **kwargs)

    def _flat_buf(self, bi, like):
        f = self._flat[bi]
        dt = self.grad_dtype or self.buckets[bi][0].dtype
        if f is None or f.device != like.device:
            f = torch.empty(self._sizes[bi], dtype=dt, device=like.device)
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
            self.launch_order.append(bi)
            self.comm.allreduce_(self._flat[bi], op="avg", wait_back=False)

    def _fp8_sites(self):
        sites = []
        for m in self.module.modules():
            d = m.__dict__.get("_fv_fp8_sites")
            if d:
                sites.extend(d[k][0] for k in sorted(d))
        return sites

    def _sync_fp8(self):
        """Every fp8 site's in-flight amax of this step, all-reduced (MAX) in ONE collective and
        rolled into every history at once (include/facevae.h fv_fp8_sites_roll): after it all
        ranks hold identical histories, so the next step's scales are global.  Sites exist
        after the first (eager) step; the device table of their pointers is rebuilt only when
        the set changes."""
        sites = self._fp8_sites()
        if not sites:
            return
        from . import _lib
        key = tuple(t.data_ptr() for t in sites)
        if key != self._fp8_key:
            dev = sites[0].device
            # the MAX all-reduce below must have the same length on every rank (a site created
            # by a forward only one rank ran would misalign it): check the counts once per set
            cnt = torch.tensor([len(sites), -len(sites)], dtype=torch.float64, device=dev)
            self.comm.allreduce_(cnt, op="max", wait_back=True)
            hi, lo = cnt.tolist()
            if hi != -lo:
                raise RuntimeError(f"DataParallel fp8: ranks hold {int(-lo)}..{int(hi)} delayed-scaling sites "
                                   f"(this rank {len(sites)}); every rank must run the same fp8 forwards")
            self._fp8_tab = torch.tensor(key, dtype=torch.int64).to(dev)
            self._fp8_amax = torch.empty(len(sites), dtype=torch.float32, device=dev)
            self._fp8_key = key
        _lib.call("fv_fp8_sites_inflight", len(sites), self._fp8_tab.data_ptr(), self._fp8_amax.data_ptr(),
                  _lib.stream())
        self.comm.allreduce_(self._fp8_amax, op="max", wait_back=True)
        _lib.call("fv_fp8_sites_roll", len(sites), self._fp8_tab.data_ptr(), self._fp8_amax.data_ptr(),
                  _lib.stream())

    def _finish(self):
        for bi, n in enumerate(self._pending):     # params that got no grad this step
            if n != 0 and n != len(self.buckets[bi]):
                raise RuntimeError("DataParallel: a bucket was only partially reduced "
                                   "(unused parameters are not supported)")
        if self._params and self._params[0].is_cuda:
            self._sync_fp8()
        self._global_fp8(False)
        if self._params:
            self.comm.fence(self._params[0].device if self._params[0].is_cuda else None)
        for bi, b in enumerate(self.buckets):
            if self._pending[bi] != 0:
                continue
            flat = self._flat[bi]
            for p in b:
                _, off = self._where[id(p)]
                v = flat[off:off + p.numel()].view_as(p)
                if v.dtype == p.dtype:
                    p.grad = v
                else:
                    p.grad.copy_(v)

    def sync_buffers(self):
        """Broadcast BN running stats / SN u, v from rank 0 (the reference's per-forward C3
        broadcast; identical under SyncBN, so done on demand, e.g. once per epoch)."""
        if self.comm is None or self.world == 1:
            return
        with torch.no_grad():
            for t in self.module.buffers():
                if t.is_floating_point():
                    self.comm.broadcast_(t.data, 0)
