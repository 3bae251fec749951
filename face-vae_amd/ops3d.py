"""torch.autograd.Functions of the AFE 3-D trunk over libfacevae (fv_conv3d_*, fv_depth_split).
No CPU fallback: every compute call goes through `_lib.call`.

Reference semantics restated (file:line in Luh1124/face-vae):
  AFE.forward's x.view(N, C, D, H, W) of the mid_conv output (models.py:941-942),
  ResBlock3D = x + NAC(NAC(x)) with ConvBlock3D "NAC" = SyncBatchNorm -> ReLU -> Conv3d 3x3x3
  (modules.py:52-56, _ResBlock 116-126, ResBlock3D 133-135; _ConvBlock 8-42).

Layout: 5-D activations are NDHWC (torch.channels_last_3d) in the storage dtype of the
compute mode.  A depth slice is then an NHWC image, so the BN statistics / apply / backward
kernels of ops.py run unchanged on the [N, C, D*H, W] channels_last alias (`as4d`).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L
from . import ops
from ._lib import call, ptr, query, stream

CL3 = torch.channels_last_3d
F32 = torch.float32


def as4d(x5: torch.Tensor) -> torch.Tensor:
    """[N, C, D, H, W] NDHWC tensor -> the [N, C, D*H, W] NHWC alias of the same memory."""
    N, C, D, H, W = x5.shape
    return x5.as_strided((N, C, D * H, W), (C * D * H * W, 1, W * C, C))


def as5d(x4: torch.Tensor, D: int) -> torch.Tensor:
    N, C, DH, W = x4.shape
    H = DH // D
    return x4.as_strided((N, C, D, H, W), (C * DH * W, 1, H * W * C, W * C, C))


def to_ndhwc(x: torch.Tensor, dtype) -> torch.Tensor:
    if not x.is_cuda:
        raise RuntimeError("facevae_amd ops run on the GPU only (HIP); got a CPU tensor")
    if x.dtype == dtype and x.is_contiguous(memory_format=CL3):
        return x
    return x.to(dtype).contiguous(memory_format=CL3)


def desc3(dtype, n, d, h, w, cin, cout):
    return L.Conv3dDesc(L.dtype_code(dtype), n, d, h, w, cin, cout)


def _dkey(d):
    return (d.dtype, d.n, d.d, d.h, d.w, d.cin, d.cout)


class Conv3dState:
    """Per-forward prepared weights of one Conv3d (wk forward, wt data gradient): the ones a
    W3PrepBatch made for this forward when they match (shape and weight version), else one
    fv_conv3d_weight_prep of its own."""

    def __init__(self, conv, d, device, need_wt):
        w = conv.weight
        if w.dtype != F32 or not w.is_contiguous():
            raise RuntimeError("conv3d weights must be contiguous fp32")
        self.conv, self.d, self.w = conv, d, w
        pre = conv.__dict__.get("_c3prep")
        if pre is not None and pre[0] == _dkey(d) and pre[1] == w._version and pre[2] is w:
            self.wk, self.wt = pre[3], pre[4]
            return
        nbytes = query("fv_conv3d_wk_bytes", ctypes.byref(d))
        if nbytes == 0:
            raise RuntimeError(f"conv3d: unsupported shape cin={d.cin} cout={d.cout}")
        self.wk = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.wt = torch.empty(nbytes, dtype=torch.uint8, device=device) if need_wt else None
        call("fv_conv3d_weight_prep", ctypes.byref(d), ptr(w), ptr(self.wk), ptr(self.wt), stream())

    def release(self):
        self.wk = None


class W3PrepBatch:
    """fv_conv3d_weight_prep_multi: the forward and data-gradient weight layouts of every conv of
    a 3-D trunk in one launch per forward (the per-conv path launched 2 per conv: 24 per AFE
    step).  Buffers persist per shape (stable addresses for graph replay); each conv finds its
    pair through `_c3prep`, checked against the shape and the weight's version."""

    def __init__(self, convs):
        self.convs = list(convs)
        self.bufs = {}

    def prep(self, d, device):
        if not self.convs:
            return
        k = _dkey(d)
        if k not in self.bufs:
            nbytes = query("fv_conv3d_wk_bytes", ctypes.byref(d))
            if nbytes == 0:
                return
            self.bufs = {k: [(torch.empty(nbytes, dtype=torch.uint8, device=device),
                              torch.empty(nbytes, dtype=torch.uint8, device=device)) for _ in self.convs]}
        pairs = self.bufs[k]
        n = len(self.convs)
        ws = [c.weight for c in self.convs]
        if any(w.dtype != F32 or not w.is_contiguous() or not w.is_cuda for w in ws):
            return
        P = ctypes.c_void_p * n
        call("fv_conv3d_weight_prep_multi", ctypes.byref(d), n, P(*[w.data_ptr() for w in ws]),
             P(*[a.data_ptr() for a, _ in pairs]), P(*[b.data_ptr() for _, b in pairs]), stream())
        for c, w, (a, b) in zip(self.convs, ws, pairs):
            c.__dict__["_c3prep"] = (k, w._version, w, a, b)


def conv3d_forward(cs: Conv3dState, x, bias, res=None, stats=False):
    """-> (y NDHWC, BN records (part, nb, bp) or None when the shape has no fused partials)."""
    d = cs.d
    y = torch.empty((d.n, d.cout, d.d, d.h, d.w), dtype=x.dtype, device=x.device, memory_format=CL3)
    rec = None
    part = None
    if stats:
        nb = query("fv_conv3d_stats_blocks", ctypes.byref(d))
        if nb > 0:
            bp = query("fv_conv3d_stats_block_pixels", ctypes.byref(d))
            part = torch.empty(nb * 2 * d.cout, dtype=F32, device=x.device)
            rec = (part, nb, bp)
    call("fv_conv3d_fwd", ctypes.byref(d), ptr(x), ptr(cs.wk), ptr(bias), ptr(res), ptr(y), ptr(part), stream())
    return y, rec


def conv3d_backward(cs: Conv3dState, x, dy, need_dx=True):
    d = cs.d
    dev = dy.device
    dw = torch.empty_like(cs.w)
    db = torch.empty(d.cout, dtype=F32, device=dev)
    nws = query("fv_conv3d_wgrad_ws_bytes", ctypes.byref(d))
    ws = ops._empty(max(nws, 4) // 4, F32, dev)
    call("fv_conv3d_bwd_weight", ctypes.byref(d), ptr(x), ptr(dy), ptr(dw), ptr(db), ptr(ws) if nws else None,
         stream())
    dx = None
    if need_dx:
        dx = torch.empty((d.n, d.cin, d.d, d.h, d.w), dtype=dy.dtype, device=dev, memory_format=CL3)
        call("fv_conv3d_bwd_data", ctypes.byref(d), ptr(dy), ptr(cs.wt), ptr(dx), stream())
    return dx, dw, db


def bn3d_stats(bn, x5, rec, training, comm):
    """BN statistics of a 5-D activation: from the producing conv's records when present,
    else one statistics pass over the tensor."""
    if not training:
        return ops.bn_finalize(bn, None, 0, False)
    N, C, D, H, W = x5.shape
    if rec is not None:
        part, nb, bp = rec
        return ops.bn_from_records(bn, part, nb, bp, N * D * H * W, C, True, comm)
    return ops.bn_from_tensor(bn, as4d(x5), True, comm)


class ResBlock3DFn(torch.autograd.Function):
    """ResBlock3D: x + NAC(NAC(x)), NAC = SyncBN -> ReLU -> Conv3d 3x3x3 (modules.py:116-135).
    The BN-apply+ReLU outputs are materialised once each; conv1's epilogue writes BN2's
    statistics records, conv2's epilogue adds the residual."""

    @staticmethod
    def forward(ctx, x, w1, b1, g1, be1, w2, b2, g2, be2, blk):
        dtype = ops.storage(blk.compute_dtype())
        xb = to_ndhwc(x, dtype)
        N, C, D, H, W = xb.shape
        training = blk.training
        comm = blk.bn_comm()
        c1, c2 = blk.conv1, blk.conv2
        r1 = bn3d_stats(blk.bn1, xb, None, training, comm)
        a1 = as5d(ops.bn_act_forward(as4d(xb), r1, 0.0, False, blk.bn1), D)
        d1 = desc3(dtype, N, D, H, W, C, c1.out_channels)
        cs1 = Conv3dState(c1, d1, x.device, True)
        t1, rec = conv3d_forward(cs1, a1, b1, stats=training)
        r2 = bn3d_stats(blk.bn2, t1, rec, training, comm)
        a2 = as5d(ops.bn_act_forward(as4d(t1), r2, 0.0, False, blk.bn2), D)
        d2 = desc3(dtype, N, D, H, W, c1.out_channels, c2.out_channels)
        cs2 = Conv3dState(c2, d2, x.device, True)
        out, _ = conv3d_forward(cs2, a2, b2, res=xb)
        cs1.release()
        cs2.release()
        ctx.blk, ctx.cs1, ctx.cs2, ctx.r1, ctx.r2, ctx.comm = blk, cs1, cs2, r1, r2, comm
        ctx.save_for_backward(x, xb, t1, a1, a2)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, xb, t1, a1, a2 = ctx.saved_tensors
        blk, cs1, cs2, r1, r2, comm = ctx.blk, ctx.cs1, ctx.cs2, ctx.r1, ctx.r2, ctx.comm
        D = xb.shape[2]
        dout = to_ndhwc(dout, xb.dtype)
        da2, dw2, db2 = conv3d_backward(cs2, a2, dout)
        dt1, dg2, dbe2 = ops.bn_act_backward(as4d(da2), as4d(t1), blk.bn2, r2, 0.0, False, comm)
        da1, dw1, db1 = conv3d_backward(cs1, a1, as5d(dt1, D))
        dxb, dg1, dbe1 = ops.bn_act_backward(as4d(da1), as4d(xb), blk.bn1, r1, 0.0, False, comm,
                                             addend=as4d(dout))
        dx = as5d(dxb, D)
        if dx.dtype != x.dtype:
            dx = dx.to(x.dtype)
        return dx, dw1, db1, dg1, dbe1, dw2, db2, dg2, dbe2, None


class DepthSplitFn(torch.autograd.Function):
    """h [N, C*D, H, W] -> h.view(N, C, D, H, W) (models.py:941-942) between the build's NHWC and
    NDHWC layouts (fv_depth_split); the backward is the inverse permutation."""

    @staticmethod
    def forward(ctx, h, C, D, dtype):
        hb, Cp = ops.to_nhwc(h, dtype)
        N, CD, H, W = h.shape
        if Cp != CD or CD != C * D:
            raise RuntimeError(f"depth split: channels {CD} != C*D = {C * D}")
        out = torch.empty((N, C, D, H, W), dtype=dtype, device=h.device, memory_format=CL3)
        call("fv_depth_split", L.dtype_code(dtype), ptr(hb), N, H * W, C, D, 0, ptr(out), stream())
        ctx.shape, ctx.dtype, ctx.hdtype = (N, C, D, H, W), dtype, h.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        N, C, D, H, W = ctx.shape
        gb = to_ndhwc(g, ctx.dtype)
        dh = torch.empty((N, C * D, H, W), dtype=ctx.dtype, device=g.device, memory_format=ops.CL)
        call("fv_depth_split", L.dtype_code(ctx.dtype), ptr(gb), N, H * W, C, D, 1, ptr(dh), stream())
        return dh.to(ctx.hdtype), None, None, None


class DepthMergeFn(torch.autograd.Function):
    """fs [N, C, D, H, W] -> fs.view(N, C*D, H, W) (models.py:1103) into the NHWC layout."""

    @staticmethod
    def forward(ctx, fs, dtype):
        fb = to_ndhwc(fs, dtype)
        N, C, D, H, W = fb.shape
        out = torch.empty((N, C * D, H, W), dtype=dtype, device=fs.device, memory_format=ops.CL)
        call("fv_depth_split", L.dtype_code(dtype), ptr(fb), N, H * W, C, D, 1, ptr(out), stream())
        ctx.shape, ctx.dtype, ctx.fdtype = (N, C, D, H, W), dtype, fs.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        N, C, D, H, W = ctx.shape
        gb, _ = ops.to_nhwc(g, ctx.dtype)
        dfs = torch.empty((N, C, D, H, W), dtype=ctx.dtype, device=g.device, memory_format=CL3)
        call("fv_depth_split", L.dtype_code(ctx.dtype), ptr(gb), N, H * W, C, D, 0, ptr(dfs), stream())
        return dfs.to(ctx.fdtype), None


def depth_split(h, C, D, mode):
    return DepthSplitFn.apply(h, C, D, ops.storage(mode))


def depth_merge(fs, mode):
    return DepthMergeFn.apply(fs, ops.storage(mode))
