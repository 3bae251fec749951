"""HIP-graph capture and replay of a whole training step (host issue).

An eager FaceVAE step issues ~270 kernels through ~400 ctypes calls, ~6 ms of host time per
step; it is hidden behind the GPU at one GPU, but it is the floor of the step as soon as the
kernels get faster.  `StepGraph` captures zero_grad -> forward -> loss -> backward -> Adam
once into a HIP graph (torch.cuda.CUDAGraph: hipStreamBeginCapture on a private stream, a
private allocator pool for every tensor the step allocates) and replays it with one
hipGraphLaunch.  Everything the step does on the host is frozen into the graph at capture:

* kernel arguments (device pointers of weights, activations and workspaces from the graph
  pool, shapes) -- fixed shapes, fixed parameter storage;
* descriptor tables (spectral-norm layers, Adam tensors) -- written once into graph-pool
  tensors at the end of the capture (`_lib.staging`, sized from the last eager step), not
  re-copied by every replay;
* the Adam step count -- moved to a device counter (`Adam.prepare_graph`,
  fv_adam_step_dev), so bias corrections advance on every replay.

Inputs are static tensors: the caller refreshes them in place (`copy_`) between replays.
Outputs are the tensors the step function returned during capture (overwritten by every
replay).

Several processes (world > 1: DataParallel bucket all-reduces, SyncBN statistics and backward
sums): the step is captured as SEGMENTS.  Every collective (and the comm-stream fence before
the optimizer) ends the current segment instead of being issued (`distributed._deferred`); the
replay runs segment 0, the first collective eagerly on its recorded tensor, segment 1, ... --
~40 graph launches and the collectives, instead of ~400 ctypes launches per step.  All segments
share one private memory pool and are replayed in capture order, so a tensor a segment writes
and the next collective reads keeps its address.  Collectives themselves are never captured
(an RCCL call inside a capture is not relied on).
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch

from . import _lib as L


def _detached(out):
    """Step outputs without their autograd graphs (tensors detached, containers rebuilt)."""
    if isinstance(out, torch.Tensor):
        return out.detach()
    if isinstance(out, dict):
        return {k: _detached(v) for k, v in out.items()}
    if isinstance(out, (list, tuple)):
        return type(out)(_detached(v) for v in out)
    return out


class SegmentRecorder:
    """Graph segments of one captured step and the eager operations between them."""

    def __init__(self):
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs = []
        self.ops = []
        self.open = False

    def begin(self):
        # relaxed: the backward's collectives (SyncBN sums, gradient buckets) run on the autograd
        # engine's device thread, so a segment is ended (and the next begun) on another thread
        # than the one that began the capture -- allowed only for relaxed-mode captures
        g = torch.cuda.CUDAGraph()
        self.stream = torch.cuda.current_stream()
        g.capture_begin(pool=self.pool, capture_error_mode="relaxed")
        self.graphs.append(g)
        self.open = True

    def cut(self, op):
        self.open = False
        self.graphs[-1].capture_end()
        self.ops.append(op)
        self.begin()

    def end(self):
        self.open = False
        self.graphs[-1].capture_end()

    def abort(self):
        """End the segment capture an exception left open (its stream -- possibly begun on the
        autograd thread -- would otherwise stay in capture mode and fail later GPU work)."""
        if self.open:
            self.open = False
            try:
                # capture_end must run with the capture stream current (the caller's except
                # clause is outside the capture's stream context)
                with torch.cuda.stream(self.stream):
                    self.graphs[-1].capture_end()
            except Exception:      # an invalidated capture still leaves capture mode; the original error is raised
                pass

    def replay(self):
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.ops):
                self.ops[i]()


class StepGraph:
    def __init__(self, step_fn: Callable, optimizers: Sequence = (), warmup: int = 2):
        if warmup < 1:
            raise ValueError("StepGraph: at least one eager warm-up step (it records the staging sizes)")
        self.step_fn = step_fn
        self.optimizers = list(optimizers)
        self.warmup = warmup
        self.graph = None
        self.out = None
        self.warm_out = None
        self._bufs = None

    def capture(self, before_capture: Callable = None):
        """Run `warmup` eager steps (real training steps) on a side stream, then capture one
        (`before_capture()` runs in between, e.g. to arm a kernel timer)."""
        from . import distributed as D
        segmented = D.get_comm() is not None and D.get_comm().world_size > 1
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for i in range(self.warmup):
                if i == self.warmup - 1:
                    L.staging.begin_record()
                # the last warm-up step's outputs (it trained), detached: a live graph of the
                # warm-up step would keep its AccumulateGrad nodes -- bound to the warm-up stream
                # -- for the captured backward, whose gradient hooks would then run on that stream
                # (a fork the segmented capture cannot end a segment across)
                self.warm_out = _detached(self.step_fn())
        cur.wait_stream(side)
        torch.cuda.synchronize()
        for o in self.optimizers:
            o.prepare_graph()
        if before_capture is not None:
            before_capture()
        self._bufs = L.staging.begin_capture()
        try:
            if segmented:
                rec = SegmentRecorder()
                cap = torch.cuda.Stream()
                cap.wait_stream(cur)
                torch.cuda.synchronize()
                D._SEGMENTS = rec
                try:
                    with torch.cuda.stream(cap):
                        rec.begin()
                        self.out = self.step_fn()
                        rec.end()
                except BaseException:
                    rec.abort()
                    raise
                finally:
                    D._SEGMENTS = None
                cur.wait_stream(cap)
                self.graph = rec
            else:
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph):
                    self.out = self.step_fn()
        finally:
            L.staging.end()
        self._tables = L.staging.keep           # the captured descriptor tables (filled once)
        if L.staging.i != len(self._bufs):
            raise RuntimeError("StepGraph: the captured step issued fewer table copies than the recorded one")
        return self

    def replay(self):
        if self.graph is None:
            raise RuntimeError("StepGraph: capture() first")
        self.graph.replay()
        for o in self.optimizers:
            o.graph_step_done()
        return self.out

    __call__ = replay
