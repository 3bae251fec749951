"""HIP-graph capture and replay of a whole training step (host issue).

An eager FaceVAE step issues ~270 kernels through ~400 ctypes calls, ~6 ms of host time per
step; it is hidden behind the GPU at one GPU, but it is the floor of the step as soon as the
kernels get faster.  `StepGraph` captures zero_grad -> forward -> loss -> backward -> Adam
once into a HIP graph (torch.cuda.CUDAGraph: hipStreamBeginCapture on a private stream, a
private allocator pool for every tensor the step allocates) and replays it with one
hipGraphLaunch.  Everything the step does on the host is frozen into the graph at capture:

* kernel arguments (device pointers of weights, activations and workspaces from the graph
  pool, shapes) -- fixed shapes, fixed parameter storage;
* descriptor tables (spectral-norm layers, Adam tensors) -- copied from pinned buffers that
  `_lib.staging` reserves for the capture from the sizes of the last eager step;
* the Adam step count -- moved to a device counter (`Adam.prepare_graph`,
  fv_adam_step_dev), so bias corrections advance on every replay.

Inputs are static tensors: the caller refreshes them in place (`copy_`) between replays.
Outputs are the tensors the step function returned during capture (overwritten by every
replay).  Single process only: RCCL collectives (DataParallel, SyncBN) stay on the eager path.
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch

from . import _lib as L


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
        if torch.distributed.is_available() and torch.distributed.is_initialized() \
                and torch.distributed.get_world_size() > 1:
            raise RuntimeError("StepGraph: single-process steps only (collectives stay eager)")
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for i in range(self.warmup):
                if i == self.warmup - 1:
                    L.staging.begin_record()
                self.warm_out = self.step_fn()     # the last warm-up step's outputs (it trained)
        cur.wait_stream(side)
        torch.cuda.synchronize()
        for o in self.optimizers:
            o.prepare_graph()
        if before_capture is not None:
            before_capture()
        self._bufs = L.staging.begin_capture()
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.graph):
                self.out = self.step_fn()
        finally:
            L.staging.end()
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
