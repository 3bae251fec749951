"""Fused multi-tensor Adam over the C-ABI (torch.optim.Adam math, logger.py:60).

state_dict layout matches torch.optim.Adam ("step", "exp_avg", "exp_avg_sq" per param), so
optimizer checkpoints interchange with the reference's Adam.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L
from ._lib import call, stream


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if weight_decay != 0.0:
            raise NotImplementedError("weight_decay (the reference uses 0)")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None))
        self._blocks = {}

    def _block_table(self, numels, device):
        key = (tuple(numels), str(device))
        t = self._blocks.get(key)
        if t is None:
            rows = []
            for i, n in enumerate(numels):
                for c in range((n + L.ADAM_CHUNK - 1) // L.ADAM_CHUNK):
                    rows.extend((i, c))
            t = torch.tensor(rows, dtype=torch.int32, device=device)
            self._blocks[key] = t
        return t

    # ------------------------------------------------------------------ HIP-graph replay
    def prepare_graph(self):
        """Before a graph capture (graph.StepGraph): the step count moves to the device (one fp64
        counter per group, advanced by the captured launch, as torch.optim.Adam(capturable=True)),
        and the group's host "step" tensors are shared so graph_step_done() is one fill."""
        self._graph = {}
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if len(self.state[p]) > 0]
            if not ps:
                continue
            n = int(self.state[ps[0]]["step"].item())
            host = torch.tensor(float(n))
            for p in ps:
                self.state[p]["step"] = host
            dev = ps[0].device
            self._graph[gi] = (torch.full((1,), float(n), dtype=torch.float64, device=dev),
                               torch.empty(2, dtype=torch.float32, device=dev), host)

    def graph_step_done(self):
        """After a replay: the host step count follows the device counter (no sync)."""
        for _, _, host in getattr(self, "_graph", {}).values():
            host.add_(1.0)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            items = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError("facevae_amd Adam: contiguous fp32 CUDA params only")
                st = self.state[p]
                if len(st) == 0:
                    if capturing:
                        raise RuntimeError("facevae_amd Adam: run an eager step before capturing a graph")
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                g = p.grad
                if not g.is_contiguous() or g.dtype != torch.float32:
                    g = g.float().contiguous()
                    p.grad = g
                items.append((p, g, st))
            if not items:
                continue
            # every param in a group advances together (logger.py steps all of them each batch)
            steps = {int(st["step"].item()) for _, _, st in items}
            if len(steps) != 1:
                raise RuntimeError("facevae_amd Adam: params of a group must share the step count")
            step = steps.pop() + 1
            dev = items[0][0].device
            descs = (L.AdamTensor * len(items))()
            for i, (p, g, st) in enumerate(items):
                descs[i] = L.AdamTensor(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                        st["exp_avg_sq"].data_ptr(), p.numel())
            blocks = self._block_table([p.numel() for p, _, _ in items], dev)
            dtab, host = L.h2d_table(bytes(descs), dev)
            if capturing:
                gs = getattr(self, "_graph", {}).get(gi)
                if gs is None:
                    raise RuntimeError("facevae_amd Adam: prepare_graph() before capturing")
                call("fv_adam_step_dev", dtab.data_ptr(), blocks.data_ptr(), blocks.numel() // 2, float(group["lr"]),
                     float(b1), float(b2), float(group["eps"]), gs[0].data_ptr(), gs[1].data_ptr(), stream())
            else:
                for _, _, st in items:
                    st["step"].fill_(float(step))
                gs = getattr(self, "_graph", {}).get(gi)
                if gs is not None:          # an eager step after a capture keeps the device count in step
                    gs[0].fill_(float(step))
                call("fv_adam_step", dtab.data_ptr(), blocks.data_ptr(), blocks.numel() // 2, float(group["lr"]),
                     float(b1), float(b2), float(group["eps"]), step, stream())
            self._keep = (dtab, host)   # keep the staging buffers alive until the launch is consumed
        return loss
