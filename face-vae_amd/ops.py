"""torch.autograd.Functions over libfacevae (the HIP C-ABI).  No CPU fallback: every
compute call goes through `_lib.call`, which raises if the library is missing or fails.

Activations between blocks are NHWC: torch tensors of logical shape [N, C, H, W] in
`torch.channels_last` memory format, dtype = the compute dtype (fp32 parity mode or bf16).
Parameters stay fp32 in the reference layout / state-dict keys.

Reference semantics restated here (file:line in Luh1124/face-vae):
  _ConvBlock "CNA"/"NAC" (modules.py:8-42), DownBlock2D (:59-70), UpBlock2D (:78-89),
  ResBlock2D (:116-130), SameBlock2D (:97-108), nn.Conv2d (models.py:934,1096,1099),
  spectral_norm (modules.py:14,32), SyncBatchNorm (modules.py:19), flatten_vae_nl
  reparameterisation (models.py:559-561), KLDivergenceLoss (losses.py:385-393),
  ReconLoss (losses.py:396-403), pixel L1 (losses.py:128,135).
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import Optional

import torch

from . import _lib as L
from ._lib import call, ptr, query, stream

CL = torch.channels_last
F32 = torch.float32
F64 = torch.float64
# fp8 compute mode (BASELINE config C5): activations and gradients stay bf16 in HBM; the 3x3
# convs the fp8 kernels support run forward and data gradient on per-tensor scaled OCP e4m3
# operands (fv_*_fp8_site: delayed scaling from a per-operand amax history, one quantize pass),
# everything else as in bf16 mode
FP8 = torch.float8_e4m3fn
# fp8: a ResBlock's bn1 backward writes the e4m3 copy of its output for the previous block's
# conv2 data gradient (ResBlockFn.backward); tests flip this off to compare with the re-quantized path
_FP8_HANDOFF = True


def storage(mode: torch.dtype) -> torch.dtype:
    """HBM dtype of activations / gradients for a compute mode."""
    return torch.bfloat16 if mode == FP8 else mode


def fp8_site(conv, which: str, device):
    """Delayed-scaling state of one fp8 operand of `conv` ("x": forward input, "dy": output
    gradient): [device buffer (fv_fp8_site_bytes), seeded flag].  Kept on the conv module, so
    the amax history spans steps (include/facevae.h, fv_quantize_fp8_site)."""
    sites = conv.__dict__.setdefault("_fv_fp8_sites", {})
    st = sites.get(which)
    if st is None or st[0].device != device:
        st = [torch.zeros(query("fv_fp8_site_bytes") // 4, dtype=torch.int32, device=device), False, []]
        sites[which] = st
    return st


# data-parallel global fp8 scaling (distributed.DataParallel at world > 1 installs its
# communicator here and turns on the deferred roll, include/facevae.h fv_fp8_set_deferred_roll)
FP8_GLOBAL = None


def _dq_snapshot(site):
    """A forward's e4m3 operand keeps a VIEW of its site's dq word for the weight gradient (no
    copy per forward: 14 copy launches per fp8 step).  Before the site is quantized again while
    such a view is still held -- a second forward through the conv before its backward, or an
    eval forward in between -- the holder gets its own copy of the value."""
    if site is None or len(site) < 3:
        return
    for ref in site[2]:
        cs = ref()
        q = getattr(cs, "x8", None) if cs is not None else None
        if q is not None and q[1].data_ptr() == site[0].data_ptr() + 18 * 4:
            cs.x8 = (q[0], q[1].clone())
    site[2].clear()


_DQ_VIEW = os.environ.get("FV_DQ_VIEW", "1") == "1"     # 0: copy the dq at every forward (A/B)


def _hold_x8(cs, x8, xdq, site):
    """cs.x8 = (x8, xdq) for the fp8 weight gradient; a dq that is the site's word is tracked
    (_dq_snapshot copies it only if the site is re-quantized before cs's backward)."""
    if not _DQ_VIEW:
        cs.x8 = (x8, xdq.clone())
        return
    cs.x8 = (x8, xdq)
    if len(site) > 2 and xdq.data_ptr() == site[0].data_ptr() + 18 * 4:
        site[2].append(weakref.ref(cs))


def quantize_fp8_site(t: torch.Tensor, site):
    """(uint8 e4m3 copy of t quantized with the site's delayed scale, dq view [1] fp32); the
    first call of a site quantizes exactly and seeds its history -- under data parallelism
    with the exact amax all-reduced (MAX) across ranks, so every rank starts from the same
    scale (the single process on the global batch)."""
    _dq_snapshot(site)
    y = _empty(t.numel(), torch.uint8, t.device)
    ws = _empty(query("fv_fp8_ws_bytes") // 4, F32, t.device)
    seeded = int(site[1])
    if not seeded and FP8_GLOBAL is not None:
        amax = _empty(1, F32, t.device)
        call("fv_fp8_amax", L.dtype_code(t.dtype), ptr(t), t.numel(), ptr(amax), ptr(ws), stream())
        FP8_GLOBAL.allreduce_(amax, op="max", wait_back=True)
        call("fv_fp8_site_seed", ptr(site[0]), ptr(amax), stream())
        seeded = 1
    call("fv_quantize_fp8_site", L.dtype_code(t.dtype), ptr(t), t.numel(), ptr(y), ptr(site[0]), seeded,
         ptr(ws), stream())
    site[1] = True
    return y, site[0][18:19].view(F32)


def pad_pow2(c: int) -> int:
    p = 8
    while p < c:
        p *= 2
    return p


def is_pow2_8(c: int) -> bool:
    return c >= 8 and (c & (c - 1)) == 0


def _empty(n, dtype, device):
    return torch.empty(int(n), dtype=dtype, device=device)


def nhwc_view(t: torch.Tensor) -> bool:
    """True if t is a dense NHWC (channels_last) tensor."""
    return t.dim() == 4 and t.is_contiguous(memory_format=CL)


def to_nhwc(x: torch.Tensor, dtype: torch.dtype):
    """x -> (buffer, channel stride): a dense NHWC tensor of `dtype` whose channel count is
    a power of two >= 8 (zero padded), as the conv kernels require."""
    if not x.is_cuda:
        raise RuntimeError("facevae_amd ops run on the GPU only (HIP); got a CPU tensor")
    N, C, H, W = x.shape
    if is_pow2_8(C):
        if x.dtype == dtype and nhwc_view(x):
            return x, C
        return x.to(dtype).contiguous(memory_format=CL), C
    cp = pad_pow2(C)
    buf = torch.empty((N, cp, H, W), dtype=dtype, device=x.device, memory_format=CL)
    x32 = x.float().contiguous()
    call("fv_nchw_to_nhwc", L.dtype_code(dtype), ptr(x32), N, C, H * W, cp, ptr(buf), stream())
    return buf, cp


def from_nhwc(buf: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """Gradient buffer (NHWC, possibly channel padded) -> tensor shaped/typed like ref."""
    N, C, H, W = ref.shape
    if buf.shape[1] == C:
        return buf.to(ref.dtype)
    out = torch.empty((N, C, H, W), dtype=F32, device=buf.device)
    call("fv_nhwc_to_nchw", L.dtype_code(buf.dtype), ptr(buf), N, C, H * W, buf.shape[1], ptr(out), stream())
    return out.to(ref.dtype)


class KernelTimer:
    """Optional HIP-event bracketing of selected conv launches (bench.py measures the dominant
    kernel's average duration live, on the stream it is launched on).  Eager launches only:
    ROCm refuses external event-record nodes inside a graph capture (hipEventRecordWithFlags(
    ..., hipEventRecordExternal) -> invalid argument on the box), so a graph-replayed bench
    times the kernel over eager steps run right after its timed region."""

    def __init__(self, match):
        self.match = match          # (kind, ConvDesc) -> bool ; kind in {"fwd", "dgrad", "wgrad"}
        self.events = {}
        self.enabled = False

    def wrap(self, kind, d, fn):
        if not (self.enabled and self.match(kind, d)):
            return fn()
        if torch.cuda.is_current_stream_capturing():
            return fn()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn()
        e1.record()
        self.events.setdefault(kind, []).append((e0, e1))
        return r

    def summary(self):
        torch.cuda.synchronize()
        return {k: [a.elapsed_time(b) for a, b in v] for k, v in self.events.items()}


TIMER: Optional[KernelTimer] = None

# Test hook (tests/test_layers_gpu.py): called after every conv launch of the model path as
# CHECK(kind, cs, **tensors) with kind in {"fwd", "dgrad", "wgrad"}, so a test can compare each
# launch, at the exact shapes and data of a real step, with a torch fp32 reference of the
# same op on the same (bf16) operands.  None in production.
CHECK = None


def _timed(kind, d, fn):
    return fn() if TIMER is None else TIMER.wrap(kind, d, fn)


def desc(dtype, n, h, w, cin, cin_valid, cout, ldy, k, ups=0, pro=0, slope=0.0, sig=0, nchw=0):
    return L.ConvDesc(L.dtype_code(dtype), n, h, w, cin, cin_valid, cout, ldy, k, int(ups), int(pro),
                      float(slope), int(sig), int(nchw))


# ----------------------------------------------------------------------------------------
# spectral norm / weights
# ----------------------------------------------------------------------------------------

def spectral_norm_fwd(w, u, v, power_iter: bool):
    rows = w.shape[0]
    cols = w.numel() // rows
    ws = _empty(query("fv_spectral_norm_ws_bytes", rows, cols) // 4 + 1, F32, w.device)
    sigma = torch.empty(1, dtype=F32, device=w.device)
    call("fv_spectral_norm_fwd", ptr(w), rows, cols, ptr(u), ptr(v), ptr(sigma), int(power_iter), ptr(ws),
         stream())
    return sigma


def spectral_norm_bwd(w, g, u, v, sigma):
    rows = w.shape[0]
    cols = w.numel() // rows
    ws = _empty(1024, F32, w.device)
    call("fv_spectral_norm_bwd", ptr(w), ptr(g), rows, cols, ptr(u), ptr(v), ptr(sigma), ptr(g), ptr(ws),
         stream())
    return g


class SNBatch:
    """One batched power iteration (4 launches) for every spectral-normed conv of a model,
    run at the start of its forward; each conv then picks up its sigma and (u, v) snapshot
    instead of running spectral_norm_fwd itself (torch/nn/utils/spectral_norm.py:62-113)."""

    def __init__(self, convs):
        self.convs = list(convs)
        self.n = len(self.convs)
        self.ws = None
        self.nb = (ctypes.c_int * 3)()
        self.tb = query("fv_spectral_norm_batch_table_bytes", self.n)
        self._host = None
        self._keep = None

    def run(self, training: bool):
        if self.n == 0:
            return
        dev = self.convs[0].weight_param().device
        sigma = torch.empty(self.n, dtype=F32, device=dev)
        snaps = [(torch.empty_like(c.weight_u), torch.empty_like(c.weight_v)) for c in self.convs]
        layers = (L.SnLayer * self.n)()
        for i, c in enumerate(self.convs):
            w = c.weight_param()
            if w.dtype != F32 or not w.is_contiguous():
                raise RuntimeError("conv weights must be contiguous fp32")
            layers[i] = L.SnLayer(w.data_ptr(), c.weight_u.data_ptr(), c.weight_v.data_ptr(),
                                  sigma.data_ptr() + 4 * i, snaps[i][0].data_ptr(), snaps[i][1].data_ptr(),
                                  w.shape[0], w.numel() // w.shape[0])
        if self.ws is None or self.ws.device != dev:
            self.ws = _empty(query("fv_spectral_norm_batch_ws_floats", ctypes.addressof(layers), self.n), F32, dev)
        host = (ctypes.c_uint8 * self.tb)()
        call("fv_spectral_norm_batch_build", ctypes.addressof(layers), self.n, ptr(self.ws), ctypes.addressof(host),
             ctypes.addressof(self.nb))
        table, hb = L.h2d_table(bytes(host), dev)
        call("fv_spectral_norm_fwd_batch", table.data_ptr(), self.n, ctypes.addressof(self.nb), int(training),
             stream())
        self._keep = (hb, table)          # alive until the launches have consumed them
        for i, c in enumerate(self.convs):
            c._sn_pre = (sigma[i:i + 1], snaps[i][0], snaps[i][1])


WPREP_MAX = 24
# fp8 weight quantization batched by WPrepBatch (tests flip it off to compare with the per-conv
# fv_conv_weight_prep_fp8 launches)
_WPREP_FP8_BATCH = os.environ.get("FV_WPREP8_BATCH", "1") != "0"


class WPrepBatch:
    """One launch (fv_conv_weight_prep_multi) for the weight re-layouts of every conv of a model
    whose last forward used a generic layout, run right after the model's SNBatch (the 1/sigma
    scales are its snapshots); each conv's ConvState then takes its prepared buffers instead of
    launching fv_conv_weight_prep (17 launches of ~7.5 us per FaceVAE step).  A conv whose
    descriptor changed since its last forward (other input shape) re-prepares itself."""

    def __init__(self, convs):
        self.convs = list(convs)

    def run(self, device):
        if _WPREP_FP8_BATCH:
            self._run_fp8(device)
        groups = {}
        for c in self.convs:
            key = getattr(c, "_fv_desc", None)
            if key is None:
                continue
            d = L.ConvDesc.from_buffer_copy(key[0])
            if not query("fv_conv_weight_prep_batchable", ctypes.byref(d)):
                continue
            sigma = None
            if c.sn:
                pre = getattr(c, "_sn_pre", None)
                if pre is None:
                    continue
                sigma = pre[0]
            groups.setdefault(d.dtype, []).append((c, d, key, sigma))
        for dt, items in groups.items():
            dtype = {L.FV_BF16: torch.bfloat16, L.FV_F32: torch.float32}[dt]
            for i0 in range(0, len(items), WPREP_MAX):
                chunk = items[i0:i0 + WPREP_MAX]
                n = len(chunk)
                descs = (L.ConvDesc * n)(*[d for _, d, _, _ in chunk])
                wp, sg, wk, wt = ((ctypes.c_void_p * n)() for _ in range(4))
                bufs = []
                for i, (c, d, key, sigma) in enumerate(chunk):
                    k = _empty(query("fv_conv_wk_elems", ctypes.byref(d)), dtype, device)
                    t = _empty(query("fv_conv_wt_elems", ctypes.byref(d)), dtype, device) if key[1] else None
                    w = c.weight_param()
                    wp[i], sg[i], wk[i], wt[i] = w.data_ptr(), ptr(sigma), k.data_ptr(), ptr(t)
                    bufs.append((c, key, k, t))
                call("fv_conv_weight_prep_multi", n, ctypes.addressof(descs), ctypes.addressof(wp),
                     ctypes.addressof(sg), ctypes.addressof(wk), ctypes.addressof(wt), stream())
                for c, key, k, t in bufs:
                    c._fv_prep = (key[0], k, t)

    def _run_fp8(self, device):
        """The e4m3 weights (+ scales) of the convs whose last forward ran fp8, in two launches
        (fv_conv_weight_prep_fp8_multi; 2 x 14 launches per fp8 FaceVAE step before)."""
        items = []
        for c in self.convs:
            key = getattr(c, "_fv_desc8", None)
            if key is None:
                continue
            sigma = None
            if c.sn:
                pre = getattr(c, "_sn_pre", None)
                if pre is None:
                    continue
                sigma = pre[0]
            items.append((c, L.ConvDesc.from_buffer_copy(key[0]), key, sigma))
        for i0 in range(0, len(items), WPREP_MAX):
            chunk = items[i0:i0 + WPREP_MAX]
            n = len(chunk)
            descs = (L.ConvDesc * n)(*[d for _, d, _, _ in chunk])
            wp, sg, wk, wt, dq = ((ctypes.c_void_p * n)() for _ in range(5))
            bufs = []
            for i, (c, d, key, sigma) in enumerate(chunk):
                k = _empty(query("fv_conv_fp8_wk_bytes", ctypes.byref(d)), torch.uint8, device)
                t = _empty(query("fv_conv_fp8_wt_bytes", ctypes.byref(d)), torch.uint8, device) if key[1] else None
                q = _empty(1, F32, device)
                wp[i], sg[i], wk[i], wt[i], dq[i] = c.weight_param().data_ptr(), ptr(sigma), k.data_ptr(), ptr(t), \
                    q.data_ptr()
                bufs.append((c, key, k, t, q))
            ws = _empty(n * query("fv_fp8_ws_bytes") // 4, F32, device)
            call("fv_conv_weight_prep_fp8_multi", n, ctypes.addressof(descs), ctypes.addressof(wp),
                 ctypes.addressof(sg), ctypes.addressof(wk), ctypes.addressof(wt), ctypes.addressof(dq), ptr(ws),
                 stream())
            for c, key, k, t, q in bufs:
                c._fv_prep8 = (key[0], k, t, q)


class ConvState:
    """Per-forward state of one conv: descriptor, prepared weights, SN snapshot.  With fp8
    (and a descriptor the fp8 kernels support) the prepared weights are e4m3 with one
    per-tensor scale (wdq) and forward / data gradient run on the fp8 kernels."""

    def __init__(self, conv, d, dtype, device, training, need_wt, fp8=False):
        self.conv = conv
        self.d = d
        w = conv.weight_param()
        if w.dtype != F32 or not w.is_contiguous():
            raise RuntimeError("conv weights must be contiguous fp32")
        self.w = w
        self.sigma = None
        if conv.sn:
            pre = getattr(conv, "_sn_pre", None)
            if pre is not None:           # computed by the model's SNBatch for this forward
                self.sigma, self.u, self.v = pre
                conv._sn_pre = None
            else:
                self.sigma = spectral_norm_fwd(w, conv.weight_u, conv.weight_v, training)
                self.u = conv.weight_u.clone()
                self.v = conv.weight_v.clone()
        self.fp8 = bool(fp8) and bool(query("fv_conv2d_fp8_supported", ctypes.byref(d)))
        if self.fp8:
            conv._fv_desc = conv._fv_prep = None
            key = (bytes(d), bool(need_wt))
            pre = getattr(conv, "_fv_prep8", None)
            conv._fv_prep8 = None
            conv._fv_desc8 = key               # what the next forward's WPrepBatch quantizes
            if pre is not None and pre[0] == key[0] and (pre[2] is not None or not need_wt):
                self.wk, self.wt, self.wdq = pre[1], (pre[2] if need_wt else None), pre[3]
                return
            self.wk = _empty(query("fv_conv_fp8_wk_bytes", ctypes.byref(d)), torch.uint8, device)
            self.wt = _empty(query("fv_conv_fp8_wt_bytes", ctypes.byref(d)), torch.uint8, device) if need_wt else None
            self.wdq = _empty(1, F32, device)
            ws = _empty(query("fv_fp8_ws_bytes") // 4, F32, device)
            call("fv_conv_weight_prep_fp8", ctypes.byref(d), ptr(w), ptr(self.sigma), ptr(self.wk), ptr(self.wt),
                 ptr(self.wdq), ptr(ws), stream())
            return
        conv._fv_desc8 = conv._fv_prep8 = None
        key = (bytes(d), bool(need_wt))
        pre = getattr(conv, "_fv_prep", None)
        conv._fv_prep = None
        conv._fv_desc = key                # what the next forward's WPrepBatch prepares
        if pre is not None and pre[0] == key[0] and (pre[2] is not None or not need_wt):
            self.wk, self.wt = pre[1], (pre[2] if need_wt else None)
            return
        self.wk = _empty(query("fv_conv_wk_elems", ctypes.byref(d)), dtype, device)
        self.wt = _empty(query("fv_conv_wt_elems", ctypes.byref(d)), dtype, device) if need_wt else None
        call("fv_conv_weight_prep", ctypes.byref(d), ptr(w), ptr(self.sigma), ptr(self.wk), ptr(self.wt),
             stream())

    def release(self):
        self.wk = None


def stats_geometry(cs: ConvState):
    """(records, pixels per record) of the BN partials the forward launch of cs writes."""
    d = ctypes.byref(cs.d)
    if cs.fp8:
        return query("fv_conv2d_fp8_stats_blocks", d), query("fv_conv2d_fp8_stats_block_pixels", d)
    return query("fv_conv2d_stats_blocks", d), query("fv_conv2d_stats_block_pixels", d)


def conv_forward(cs: ConvState, x, bias, pro=None, res=None, y=None, stats=False, x8=None):
    """x8: (e4m3 copy of x, dq) already written by x's producer (bn_act_forward_q8), fp8 mode."""
    d = cs.d
    part = None
    if stats:
        nb, _ = stats_geometry(cs)
        part = _empty(nb * 2 * d.cout, F32, x.device)
    psc, psh = (pro if pro is not None else (None, None))
    if cs.fp8:
        site = fp8_site(cs.conv, "x", x.device)
        x8, xdq = x8 if x8 is not None else quantize_fp8_site(x, site)
        # the e4m3 operand stays for the fp8 weight gradient; its dq is the site's word 18,
        # which the site's next quantization rewrites (a second forward through this conv, or
        # an eval forward, before this backward): _dq_snapshot copies it then
        _hold_x8(cs, x8, xdq, site)
        _timed("fwd", d, lambda: call("fv_conv2d_fwd_fp8_site", ctypes.byref(d), ptr(x8), ptr(site[0]), ptr(cs.wk),
                                      ptr(cs.wdq), ptr(bias), ptr(res), ptr(y), ptr(part), stream()))
        if CHECK is not None:
            CHECK("fwd", cs, x=x, bias=bias, pro=pro, res=res, y=y, q8=(x8, xdq))
        return part
    _timed("fwd", d, lambda: call("fv_conv2d_fwd", ctypes.byref(d), ptr(x), ptr(cs.wk), ptr(bias), ptr(psc),
                                  ptr(psh), ptr(res), ptr(y), ptr(part), stream()))
    if CHECK is not None:
        CHECK("fwd", cs, x=x, bias=bias, pro=pro, res=res, y=y)
    return part


# store-pass reductions (include/facevae.h, fv_store_reduce)
def sr_records(d, dgrad):
    """(records, pixels per record) of the store-pass reduction of a launch, or None."""
    bp = ctypes.c_int(0)
    nrec = query("fv_conv2d_sr_records", ctypes.byref(d), int(dgrad), ctypes.byref(bp))
    return (nrec, bp.value) if nrec > 0 else None


class BNRecords:
    """BN-backward sums of a BN output gradient, reduced in the dgrad that produced it."""
    __slots__ = ("part", "nb", "bp", "dx")

    def __init__(self, part, nb, bp, dx):
        self.part, self.nb, self.bp, self.dx = part, nb, bp, dx


def _dgrad_bnred(cs, dy, dx, bnred):
    """Data gradient with the BN-backward sums of `bnred` = (bn, BNResult, bn input y, slope)
    fused into its store pass; -> BNRecords, or None (then dx is not written)."""
    d = cs.d
    if bnred is None or cs.fp8 or d.upsample or d.dtype != L.FV_BF16:
        return None
    geo = sr_records(d, True)
    if geo is None:
        return None
    bn, r, ybn, slope = bnred
    if r.count == 0 and r.stats is None:          # eval-mode statistics: no batch sums needed
        return None
    nb, bp = geo
    part = _empty(nb * 2 * d.cin, F32, dy.device)
    sr = L.StoreReduce(2, ptr(part), ptr(ybn), ptr(r.mean), ptr(r.invstd), ptr(bn.weight), ptr(bn.bias),
                       float(slope))
    _timed("dgrad", d, lambda: call("fv_conv2d_bwd_data_sr", ctypes.byref(d), ptr(dy), d.cout, ptr(cs.wt), ptr(dx),
                                    ctypes.byref(sr), stream()))
    return BNRecords(part, nb, bp, dx)


def _wgrad(cs: ConvState, x, dy, ldd, pro, need_db):
    d = cs.d
    dev = dy.device
    slab = _empty(query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), F32, dev)
    bslab = _empty(query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), F32, dev) if need_db else None
    psc, psh = (pro if pro is not None else (None, None))
    _timed("wgrad", d, lambda: call("fv_conv2d_bwd_weight", ctypes.byref(d), ptr(x), ptr(psc), ptr(psh), ptr(dy),
                                    ldd, ptr(slab), ptr(bslab), stream()))
    return _wgrad_finish(cs, x, dy, ldd, pro, need_db, slab, bslab)


def _wgrad_fp8(cs: ConvState, x, dy, ldd, need_db, dy8):
    d = cs.d
    dev = dy.device
    x8, xdq = cs.x8
    dy8_, dydq = dy8
    slab = _empty(query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), F32, dev)
    bslab = _empty(query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), F32, dev) if need_db else None
    _timed("wgrad", d, lambda: call("fv_conv2d_bwd_weight_fp8", ctypes.byref(d), ptr(x8), ptr(xdq), ptr(dy8_), ptr(dydq),
                                    ptr(slab), ptr(bslab), stream()))
    cs.x8 = None
    return _wgrad_finish(cs, x, dy, ldd, None, need_db, slab, bslab, q8=(x8, xdq, dy8_, dydq))


def _wgrad_finish(cs: ConvState, x, dy, ldd, pro, need_db, slab, bslab, q8=None):
    d = cs.d
    dev = dy.device
    dw = torch.empty_like(cs.w)
    db = torch.empty(d.cout, dtype=F32, device=dev) if need_db else None
    # the fp8 weight gradient's slabs (images per split of its own) have their own reduce
    call("fv_conv2d_wgrad_fp8_reduce" if q8 is not None else "fv_conv2d_wgrad_reduce", ctypes.byref(d), ptr(slab),
         ptr(bslab), ptr(dw), ptr(db), stream())
    if CHECK is not None:
        CHECK("wgrad", cs, x=x, dy=dy, ldd=ldd, dw=dw, db=db, pro=pro, q8=q8)
    if cs.conv.sn and not (_sn_defer_ok(cs) and _sn_defer(cs)):
        spectral_norm_bwd(cs.w, dw, cs.u, cs.v, cs.sigma)
    return dw, db


# Spectral-norm backward terms batched at the end of backward:
# instead of two launches per SN conv (<g, w> partials, then the rank-1 update), one
# fv_spectral_norm_bwd_multi pair for every SN conv of the backward pass, applied in place to
# the parameters' .grad from an autograd final callback.  Only in a single process (data-parallel
# hooks all-reduce each gradient as it is accumulated, so the term must be in it by then) and
# only for parameters whose .grad was None (AccumulateGrad then holds exactly this gradient).
_SN_BATCH = True          # tests/test_graph_gpu.py flips it to compare with the per-conv launches
_SN_DEFER = {"items": [], "armed": False, "stream": None}


def _sn_defer_ok(cs: ConvState) -> bool:
    if not _SN_BATCH or cs.w.grad is not None:
        return False
    if torch.distributed.is_available() and torch.distributed.is_initialized() \
            and torch.distributed.get_world_size() > 1:
        return False
    return True


def _sn_flush():
    items, st = _SN_DEFER["items"], _SN_DEFER["stream"]
    _SN_DEFER.update(items=[], armed=False, stream=None)
    layers = [(w, u, v, sig) for w, u, v, sig in items if w.grad is not None]
    if not layers:
        return
    with torch.cuda.stream(st):
        for i0 in range(0, len(layers), 24):
            chunk = layers[i0:i0 + 24]
            arr = (L.SnBwdLayer * len(chunk))()
            for i, (w, u, v, sig) in enumerate(chunk):
                g = w.grad
                if g.dtype != F32 or not g.is_contiguous():
                    raise RuntimeError("spectral-norm backward: fp32 contiguous gradient expected")
                arr[i] = L.SnBwdLayer(w.data_ptr(), g.data_ptr(), u.data_ptr(), v.data_ptr(), sig.data_ptr(),
                                      w.shape[0], w.numel() // w.shape[0])
            ws = _empty(256 * len(chunk), F32, chunk[0][0].device)
            call("fv_spectral_norm_bwd_multi", len(chunk), ctypes.addressof(arr), ptr(ws), stream())


def _sn_defer(cs: ConvState) -> bool:
    """Queue cs's spectral-norm term for the end of this backward pass (applied on the current
    compute stream); False (caller applies it now) outside a backward pass."""
    if any(w is cs.w for w, _, _, _ in _SN_DEFER["items"]):
        raise RuntimeError("spectral-norm backward batching: a conv used twice in one backward pass")
    if not _SN_DEFER["armed"]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(_sn_flush)
        except RuntimeError:         # not inside a backward pass
            return False
        _SN_DEFER["armed"] = True
        _SN_DEFER["stream"] = torch.cuda.current_stream(cs.w.device)
    _SN_DEFER["items"].append((cs.w, cs.u, cs.v, cs.sigma))
    return True


def conv_backward(cs: ConvState, x, dy, ldd, pro=None, need_dx=True, need_db=True, bnred=None, want_recs=False,
                  dy8=None):
    """-> (dx at the conv input resolution (upsample folded back), dW (param layout), db
    [, BNRecords or None when want_recs]).  dy8: (e4m3 copy of dy, dq) from dy's producer.
    fp8: the weight gradient runs on the e4m3 x (kept by the forward) and dy as well, when the
    shape allows (fv_conv2d_wgrad_fp8_supported)."""
    if cs.fp8 and getattr(cs, "x8", None) is not None and query("fv_conv2d_wgrad_fp8_supported", ctypes.byref(cs.d)):
        site = fp8_site(cs.conv, "dy", dy.device)
        dy8 = dy8 if dy8 is not None else quantize_fp8_site(dy, site)
        dw, db = _wgrad_fp8(cs, x, dy, ldd, need_db, dy8)
    else:
        if x.numel() == 0 or (dy.numel() == 0 and dy8 is None):
            # q8_only: the activation / gradient exists only as its e4m3 copy, which the first
            # backward consumed (cs.x8 released); a second backward (retain_graph=True) would
            # read the 0-element placeholder
            raise RuntimeError("conv backward: the bf16 operand of this fp8 conv was never materialised "
                               "(FV_Q8_ONLY) and its e4m3 copy was released by an earlier backward; "
                               "backward through an fp8 ResBlock runs once (no retain_graph)")
        dw, db = _wgrad(cs, x, dy, ldd, pro, need_db)
    dx, recs = _dgrad(cs, dy, ldd, need_dx, bnred, dy8)
    return (dx, dw, db, recs) if want_recs else (dx, dw, db)


def _dgrad(cs: ConvState, dy, ldd, need_dx, bnred, dy8=None):
    """Data gradient of cs -> (dx or None, BNRecords or None)."""
    d = cs.d
    dev = dy.device
    if not need_dx:
        return None, None
    if cs.fp8:
        site = fp8_site(cs.conv, "dy", dy.device)
        dy8, dydq = dy8 if dy8 is not None else quantize_fp8_site(dy, site)
        dx = torch.empty((d.n, d.cin, d.h, d.w), dtype=dy.dtype, device=dev, memory_format=CL)
        _timed("dgrad", d, lambda: call("fv_conv2d_bwd_data_fp8_site", ctypes.byref(d), ptr(dy8), ptr(site[0]),
                                        ptr(cs.wt), ptr(cs.wdq), ptr(dx), stream()))
        if CHECK is not None:
            CHECK("dgrad", cs, dy=dy, ldd=ldd, dx=dx, q8=(dy8, dydq))
        return dx, None
    if d.upsample and query("fv_conv2d_dgrad_lowres", ctypes.byref(d)):
        # gradient of the upsample's (low-res) input in one stride-2 pass
        dx = torch.empty((d.n, d.cin, d.h // 2, d.w // 2), dtype=dy.dtype, device=dev, memory_format=CL)
        _timed("dgrad", d, lambda: call("fv_conv2d_bwd_data", ctypes.byref(d), ptr(dy), ldd, ptr(cs.wt), ptr(dx),
                                        stream()))
    else:
        dx = torch.empty((d.n, d.cin, d.h, d.w), dtype=dy.dtype, device=dev, memory_format=CL)
        recs = _dgrad_bnred(cs, dy, dx, bnred) if ldd == d.cout else None
        if recs is not None:
            if CHECK is not None:
                CHECK("dgrad", cs, dy=dy, ldd=ldd, dx=dx)
            return dx, recs
        _timed("dgrad", d, lambda: call("fv_conv2d_bwd_data", ctypes.byref(d), ptr(dy), ldd, ptr(cs.wt), ptr(dx),
                                        stream()))
        if d.upsample:
            src = torch.empty((d.n, d.cin, d.h // 2, d.w // 2), dtype=dy.dtype, device=dev, memory_format=CL)
            call("fv_upsample2x_bwd", L.dtype_code(dy.dtype), ptr(dx), d.n, d.h // 2, d.w // 2, d.cin, ptr(src),
                 stream())
            dx = src
    if CHECK is not None:
        CHECK("dgrad", cs, dy=dy, ldd=ldd, dx=dx)
    return dx, None


# ----------------------------------------------------------------------------------------
# batch norm
# ----------------------------------------------------------------------------------------

class BNResult:
    """Per-forward BN state: save_mean / save_invstd / fused (scale, shift), and the element
    count -- a host int in a single process, or `stats` (the all-reduced fp64 [3][C] record
    whose row 0 is the global count) under SyncBN."""
    __slots__ = ("mean", "invstd", "scale", "shift", "count", "stats")


def _bn_result(C, dev, count, stats=None):
    r = BNResult()
    r.mean = torch.empty(C, dtype=F32, device=dev)
    r.invstd = torch.empty(C, dtype=F32, device=dev)
    r.scale = torch.empty(C, dtype=F32, device=dev)
    r.shift = torch.empty(C, dtype=F32, device=dev)
    r.count = count
    r.stats = stats
    return r


def _running(bn, training):
    """(running_mean, running_var, num_batches_tracked) pointers the finalize updates/reads."""
    upd = training and bn.track_running_stats
    use = upd or not training
    nbt = bn.num_batches_tracked if (upd and bn.num_batches_tracked is not None) else None
    return (ptr(bn.running_mean if use else None), ptr(bn.running_var if use else None), ptr(nbt))


def bn_finalize(bn, stats, count, training):
    """stats [3][C] fp64 (already all-reduced for SyncBN) -> BNResult; updates running stats
    and num_batches_tracked (torch/nn/modules/batchnorm.py:744-840)."""
    C = bn.num_features
    r = _bn_result(C, bn.weight.device, count, stats)
    rm, rv, nbt = _running(bn, training)
    call("fv_bn_finalize", ptr(stats), C, ptr(bn.weight), ptr(bn.bias), float(bn.eps), float(bn.momentum),
         int(training), rm, rv, nbt, ptr(r.mean), ptr(r.invstd), ptr(r.scale), ptr(r.shift), stream())
    return r


def _sync(stats, comm):
    """SyncBN all-reduce (sum) of an fp64 record, in stream order (distributed.py)."""
    if comm is not None:
        comm.allreduce_(stats, op="sum", wait_back=True)


def bn_from_partials(bn, part, cs, training, comm):
    d = cs.d
    nb, bp = stats_geometry(cs)
    return bn_from_records(bn, part, nb, bp, d.n * d.h * d.w, d.cout, training, comm)


def bn_from_records(bn, part, nb, bp, P, C, training, comm):
    """BN statistics from nb (sum, sum of squares) records of bp pixels each (P in total)."""
    dev = part.device
    ws = _empty(query("fv_bn_ws_bytes", C) // 8, F64, dev)
    if comm is None:
        # single process: statistics + finalize in two launches
        r = _bn_result(C, dev, P)
        rm, rv, nbt = _running(bn, True)
        call("fv_bn_stats_finalize_partials", ptr(part), nb, bp, P, C, ptr(bn.weight), ptr(bn.bias), float(bn.eps),
             float(bn.momentum), rm, rv, nbt, ptr(r.mean), ptr(r.invstd), ptr(r.scale), ptr(r.shift), ptr(ws),
             stream())
        return r
    stats = torch.empty(3 * C, dtype=F64, device=dev)
    call("fv_bn_stats_from_partials", ptr(part), nb, bp, P, C, ptr(stats), ptr(ws), stream())
    _sync(stats, comm)                      # row 0 (count) is summed too: the global count
    return bn_finalize(bn, stats, None, training)


def bn_from_tensor(bn, x, training, comm):
    N, C, H, W = x.shape
    if not training:
        return bn_finalize(bn, None, 0, False)
    ws = _empty(query("fv_bn_ws_bytes", C) // 8, F64, x.device)
    if comm is None:
        r = _bn_result(C, x.device, N * H * W)
        rm, rv, nbt = _running(bn, True)
        call("fv_bn_stats_finalize_tensor", L.dtype_code(x.dtype), ptr(x), N * H * W, C, C, ptr(bn.weight),
             ptr(bn.bias), float(bn.eps), float(bn.momentum), rm, rv, nbt, ptr(r.mean), ptr(r.invstd), ptr(r.scale),
             ptr(r.shift), ptr(ws), stream())
        return r
    stats = torch.empty(3 * C, dtype=F64, device=x.device)
    call("fv_bn_stats_tensor", L.dtype_code(x.dtype), ptr(x), N * H * W, C, C, ptr(stats), ptr(ws), stream())
    _sync(stats, comm)
    return bn_finalize(bn, stats, None, True)


def bn_act_forward(y, r: BNResult, slope, pool, bn=None):
    N, C, H, W = y.shape
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    out = torch.empty((N, C, Ho, Wo), dtype=y.dtype, device=y.device, memory_format=CL)
    call("fv_bn_act_fwd", L.dtype_code(y.dtype), ptr(y), N, H, W, C, C, ptr(r.scale), ptr(r.shift), float(slope),
         int(pool), ptr(out), stream())
    if CHECK is not None:
        CHECK("bn_fwd", bn, y=y, r=r, slope=slope, pool=pool, out=out)
    return out


def _q8_ok(site, y, pool, bn=None):
    """The fused fp8 copy applies: a seeded site (the exact first call stays a separate pass),
    bf16 storage, no pooling, affine BN."""
    return (site is not None and site[1] and not pool and y.dtype == torch.bfloat16
            and (bn is None or (bn.weight is not None and bn.bias is not None)))


_Q8_ONLY = os.environ.get("FV_Q8_ONLY", "1") == "1"   # tests/test_fp8_gpu.py flips it to compare with the bf16-writing passes
# fp8 ResBlock conv2: store-pass BN statistics of the residual-added output in the e4m3 conv's
# epilogue (fv_conv2d_fwd_fp8_site_sr) instead of a tensor_stats pass; FV_FP8_SR=0 for A/B
FP8_SR = os.environ.get("FV_FP8_SR", "1") == "1"


def q8_only(cs: ConvState) -> bool:
    """True when conv cs reads its input x (or its output gradient dy) ONLY as the e4m3 copy:
    fp8 forward, fp8 data gradient and fp8 weight gradient (fv_conv2d_wgrad_fp8_supported), no
    checker attached.  The producing BN pass then writes the e4m3 copy alone, not the bf16
    tensor beside it (one bf16 write of the activation less per pass)."""
    return _Q8_ONLY and CHECK is None and cs.fp8 and bool(query("fv_conv2d_wgrad_fp8_supported", ctypes.byref(cs.d)))


def bn_act_forward_q8(y, r: BNResult, slope, bn, site, only8=False):
    """bn_act_forward for an fp8 consumer: -> (out, (e4m3 copy, dq) or None).  With a seeded
    delayed-scaling site the pass writes the consumer's fp8 operand beside `out`
    (fv_bn_act_fwd_q8), so the conv needs no quantize pass of its own.  only8 (q8_only(consumer)):
    the e4m3 copy alone -- `out` is then a 0-element placeholder of the right dtype / device."""
    if not _q8_ok(site, y, False):
        return bn_act_forward(y, r, slope, False, bn), None
    _dq_snapshot(site)
    N, C, H, W = y.shape
    n = N * C * H * W
    if only8:
        out = torch.empty(0, dtype=y.dtype, device=y.device)
    else:
        out = torch.empty((N, C, H, W), dtype=y.dtype, device=y.device, memory_format=CL)
    out8 = _empty(n, torch.uint8, y.device)
    call("fv_bn_act_fwd_q8", L.dtype_code(y.dtype), ptr(y), N, H, W, C, ptr(r.scale), ptr(r.shift), float(slope),
         None if only8 else ptr(out), ptr(out8), ptr(site[0]), stream())
    if CHECK is not None:
        CHECK("bn_fwd", bn, y=y, r=r, slope=slope, pool=False, out=out)
    return out, (out8, site[0][18:19].view(F32))


def bn_backward_is_local(r: BNResult, comm) -> bool:
    """True when this BN's backward needs no collective: no communicator, or eval-mode
    statistics (running mean / var, count 0, no all-reduced record) -- the normalisation is
    then a fixed per-channel affine map, so dx = gamma * invstd * g on every rank and dgamma /
    dbeta are this rank's sums (averaged later with the other gradients), exactly as torch's
    SyncBatchNorm falls back to batch_norm in eval mode (torch/nn/modules/batchnorm.py:790-826)."""
    return comm is None or (r.count == 0 and r.stats is None)


def bn_act_backward(dout, y, bn, r: BNResult, slope, pool, comm, addend=None, need_dx=True, recs=None, q8=None,
                    only8=False):
    """-> (dx of the BN input, dgamma, dbeta).  recs: the BN-backward sums already reduced by
    the dgrad that produced dout (BNRecords), replacing the reduce pass.  q8: the delayed-scaling
    site of an fp8 data gradient consuming dx -> (dx, dgamma, dbeta, (e4m3 copy of dx, dq) or
    None), the copy written by the apply pass itself (fv_bn_act_bwd_apply_q8); only8
    (q8_only(consumer)): that copy alone, dx a 0-element placeholder."""
    N, C, H, W = y.shape
    dev = y.device
    dc = L.dtype_code(y.dtype)
    if bn_backward_is_local(r, comm):
        comm = None
    ws = _empty(query("fv_bn_ws_bytes", C) // 8, F64, dev)
    dg = torch.empty(C, dtype=F32, device=dev)
    dbt = torch.empty(C, dtype=F32, device=dev)
    k = torch.empty(2 * C, dtype=F32, device=dev)
    if recs is not None and not pool and recs.dx.data_ptr() == dout.data_ptr():
        P = N * H * W
        if comm is None:
            call("fv_bn_bwd_from_records", ptr(recs.part), recs.nb, recs.bp, P, C, int(r.count), ptr(dg), ptr(dbt),
                 ptr(k), None, ptr(ws), stream())
        else:
            red = torch.empty(2 * C, dtype=F64, device=dev)
            call("fv_bn_bwd_from_records", ptr(recs.part), recs.nb, recs.bp, P, C, 0, ptr(dg), ptr(dbt), None,
                 ptr(red), ptr(ws), stream())
            if need_dx:
                _sync(red, comm)
                call("fv_bn_bwd_finalize_dev", ptr(red), C, ptr(r.stats), None, None, ptr(k), stream())
    elif comm is None:
        # eval mode (running statistics, count 0): the normalisation is a fixed affine map, so
        # the batch-statistics terms k vanish and dx = gamma * invstd * g
        evalm = r.count == 0 and r.stats is None
        call("fv_bn_act_bwd_reduce_finalize", dc, ptr(dout), ptr(y), N, H, W, C, C, ptr(r.mean), ptr(r.invstd),
             ptr(bn.weight), ptr(bn.bias), float(slope), int(pool), 1 if evalm else int(r.count), ptr(dg), ptr(dbt),
             ptr(k), ptr(ws), stream())
        if evalm:
            k.zero_()
    else:
        red = torch.empty(2 * C, dtype=F64, device=dev)
        call("fv_bn_act_bwd_reduce", dc, ptr(dout), ptr(y), N, H, W, C, C, ptr(r.mean), ptr(r.invstd),
             ptr(bn.weight), ptr(bn.bias), float(slope), int(pool), ptr(red), ptr(ws), stream())
        # dgamma / dbeta from this rank's sums (torch SyncBatchNorm: batch_norm_backward_reduce
        # is local, only sum_dy / sum_dy_xmu are all-reduced, and only when the input needs a
        # gradient -- _functions.py); the data-parallel gradient average then yields the
        # global-batch value.  dx uses the global sums over the global count (stats row 0).
        call("fv_bn_bwd_finalize", ptr(red), C, 0, ptr(dg), ptr(dbt), None, stream())
        if need_dx:
            _sync(red, comm)
            call("fv_bn_bwd_finalize_dev", ptr(red), C, ptr(r.stats), None, None, ptr(k), stream())
    dx = q = None
    if need_dx:
        q8ok = _q8_ok(q8, y, pool, bn)
        if q8ok and only8:
            dx = torch.empty(0, dtype=y.dtype, device=dev)
        else:
            dx = torch.empty((N, C, H, W), dtype=y.dtype, device=dev, memory_format=CL)
        if q8ok:
            dx8 = _empty(N * C * H * W, torch.uint8, dev)
            call("fv_bn_act_bwd_apply_q8", dc, ptr(dout), ptr(y), N, H, W, C, ptr(r.mean), ptr(r.invstd),
                 ptr(bn.weight), ptr(bn.bias), float(slope), ptr(k), ptr(addend), None if only8 else ptr(dx),
                 ptr(dx8), ptr(q8[0]), stream())
            q = (dx8, q8[0][18:19].view(F32))
        else:
            call("fv_bn_act_bwd_apply", dc, ptr(dout), ptr(y), N, H, W, C, C, ptr(r.mean), ptr(r.invstd),
                 ptr(bn.weight), ptr(bn.bias), float(slope), int(pool), ptr(k), ptr(addend), ptr(dx), stream())
    if CHECK is not None and comm is None:
        CHECK("bn_bwd", bn, dout=dout, y=y, r=r, slope=slope, pool=pool, addend=addend, dx=dx, dg=dg, dbt=dbt)
    return (dx, dg, dbt, q) if q8 is not None else (dx, dg, dbt)


def grad_in(g: torch.Tensor, dtype) -> torch.Tensor:
    return g.to(dtype).contiguous(memory_format=CL)


# ----------------------------------------------------------------------------------------
# autograd Functions
# ----------------------------------------------------------------------------------------

class ConvBNActFn(torch.autograd.Function):
    """CNA block: conv -> BN -> act [-> AvgPool2d(2)], optional nearest-x2 upsample in front
    (ConvBlock2D "CNA", DownBlock2D, UpBlock2D, SameBlock2D)."""

    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, blk):
        mode = blk.compute_dtype()
        dtype = storage(mode)
        conv, bn = blk.conv, blk.bn
        xb, cin_pad = to_nhwc(x, dtype)
        N, _, Hi, Wi = x.shape
        H, W = (2 * Hi, 2 * Wi) if blk.upsample else (Hi, Wi)
        cout = conv.out_channels
        if cout % 8:
            raise RuntimeError("CNA block output channels must be a multiple of 8")
        training = blk.training
        d = desc(dtype, N, H, W, cin_pad, conv.in_channels, cout, cout, conv.kernel_size, ups=blk.upsample)
        cs = ConvState(conv, d, dtype, x.device, training, need_wt=ctx.needs_input_grad[0], fp8=mode == FP8)
        y = torch.empty((N, cout, H, W), dtype=dtype, device=x.device, memory_format=CL)
        part = conv_forward(cs, xb, bias, y=y, stats=training)
        comm = blk.bn_comm()
        r = bn_from_partials(bn, part, cs, True, comm) if training else bn_finalize(bn, None, 0, False)
        z = bn_act_forward(y, r, blk.slope, blk.pool, bn)
        cs.release()
        ctx.blk, ctx.cs, ctx.r, ctx.comm = blk, cs, r, comm
        # z = act(BN(y)): a single consumer conv may reduce this BN's backward sums in the store
        # pass of its data gradient (holder["recs"], read back in backward below)
        ctx.holder = {"bn": bn, "r": r, "y": y, "slope": blk.slope, "pool": blk.pool, "nuse": 0}
        blk._fv_holder = ctx.holder if training else None
        ctx.src = _claim_bnsrc(x, xb)
        ctx.save_for_backward(x, xb, y)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, xb, y = ctx.saved_tensors
        blk, cs, r = ctx.blk, ctx.cs, ctx.r
        dz = grad_in(dz, y.dtype)
        recs = ctx.holder.get("recs") if ctx.holder["nuse"] == 1 else None
        # fp8 conv (Generator.in_conv): the BN backward apply writes the e4m3 copy of dy its data
        # and weight gradients consume (no quantize pass over dy; r6)
        q8 = fp8_site(cs.conv, "dy", y.device) if cs.fp8 and not blk.pool else None
        out = bn_act_backward(dz, y, blk.bn, r, blk.slope, blk.pool, ctx.comm, recs=recs, q8=q8)
        dy, dg, dbt = out[:3]
        dxb, dw, db, recs_in = conv_backward(cs, xb, dy, y.shape[1], need_dx=ctx.needs_input_grad[0],
                                             bnred=_bnred_of(ctx.src), want_recs=True,
                                             dy8=out[3] if q8 is not None else None)
        if ctx.src is not None:
            ctx.src["recs"] = recs_in
        dx = from_nhwc(dxb, x) if dxb is not None else None
        return dx, dw, db, dg, dbt, None


def _claim_bnsrc(x, xb):
    """The BN-source holder of x (set by the producing CNA block) when this Function's data
    gradient will be x's whole gradient in the producer's layout; counts the consumers."""
    src = getattr(x, "_fv_bnsrc", None)
    if src is None or src[1] != x._version:
        return None
    h = src[0]
    h["nuse"] += 1
    return h if (xb is x and not h["pool"]) else None


def _bnred_of(src):
    return None if src is None or src["nuse"] != 1 else (src["bn"], src["r"], src["y"], src["slope"])


class ResBlockFn(torch.autograd.Function):
    """ResBlock2D: x + NAC(NAC(x)), NAC = BN -> ReLU -> conv3x3 (modules.py:116-130).  The
    BN-apply+ReLU output of each NAC is materialised once (one HBM pass, written with its e4m3
    copy in fp8 mode).  (Applying BN + ReLU in the convs' operand staging instead -- "option A",
    rounds 4-5 -- measured slower twice and was removed in round 6)  The residual
    add runs in conv2's epilogue."""

    @staticmethod
    def forward(ctx, x, w1, b1, g1, be1, w2, b2, g2, be2, blk):
        mode = blk.compute_dtype()
        dtype = storage(mode)
        xb, C = to_nhwc(x, dtype)
        if C != x.shape[1]:
            raise RuntimeError("ResBlock2D channels must be a power of two >= 8")
        N, _, H, W = x.shape
        training = blk.training
        comm = blk.bn_comm()
        c1, c2 = blk.conv1, blk.conv2
        rec = getattr(x, "_fv_bnrec", None)
        if training and rec is not None and rec[3] == x._version and xb is x:
            # statistics of x reduced in the previous block's conv2 store pass (post-residual)
            r1 = bn_from_records(blk.bn1, rec[0], rec[1], rec[2], N * H * W, C, True, comm)
        else:
            r1 = bn_from_tensor(blk.bn1, xb, training, comm)
        d1 = desc(dtype, N, H, W, C, C, C, C, c1.kernel_size)
        cs1 = ConvState(c1, d1, dtype, x.device, training, True, fp8=mode == FP8)
        # fp8 convs: the BN pass writes the conv's e4m3 operand beside its bf16 output
        a1, q1 = bn_act_forward_q8(xb, r1, 0.0, blk.bn1, fp8_site(c1, "x", x.device) if cs1.fp8 else None,
                                   only8=q8_only(cs1))
        t1 = torch.empty_like(xb)
        part = conv_forward(cs1, a1, b1, y=t1, stats=training, x8=q1)
        r2 = bn_from_partials(blk.bn2, part, cs1, True, comm) if training else bn_finalize(blk.bn2, None, 0, False)
        d2 = desc(dtype, N, H, W, C, C, C, C, c2.kernel_size)
        cs2 = ConvState(c2, d2, dtype, x.device, training, True, fp8=mode == FP8)
        a2, q2 = bn_act_forward_q8(t1, r2, 0.0, blk.bn2, fp8_site(c2, "x", x.device) if cs2.fp8 else None,
                                   only8=q8_only(cs2))
        out = torch.empty_like(xb)
        geo = sr_records(d2, False) if training and (not cs2.fp8 or FP8_SR) else None
        if geo is not None:
            # out = x + conv2(.) with its (sum, sum of squares) reduced in the store pass: the
            # next ResBlock's bn1 statistics without a pass over out (ResBlock2D.forward hands
            # them on); in fp8 mode the e4m3 conv's staged epilogue does the same (r6)
            part = _empty(geo[0] * 2 * C, F32, x.device)
            sr = L.StoreReduce(1, ptr(part), None, None, None, None, None, 0.0)
            if cs2.fp8:
                site = fp8_site(c2, "x", x.device)
                x8, xdq = q2 if q2 is not None else quantize_fp8_site(a2, site)
                _hold_x8(cs2, x8, xdq, site)
                _timed("fwd", d2, lambda: call("fv_conv2d_fwd_fp8_site_sr", ctypes.byref(d2), ptr(x8), ptr(site[0]),
                                               ptr(cs2.wk), ptr(cs2.wdq), ptr(b2), ptr(xb), ptr(out),
                                               ctypes.byref(sr), stream()))
                if CHECK is not None:
                    CHECK("fwd", cs2, x=a2, bias=b2, pro=None, res=xb, y=out, q8=(x8, xdq))
            else:
                _timed("fwd", d2, lambda: call("fv_conv2d_fwd_sr", ctypes.byref(d2), ptr(a2), ptr(cs2.wk), ptr(b2),
                                               ptr(xb), ptr(out), ctypes.byref(sr), stream()))
                if CHECK is not None:
                    CHECK("fwd", cs2, x=a2, bias=b2, pro=None, res=xb, y=out)
            blk._fv_out_rec = (part, geo[0], geo[1])
        else:
            conv_forward(cs2, a2, b2, res=xb, y=out, x8=q2)
            blk._fv_out_rec = None
        cs1.release()
        cs2.release()
        # fp8: the gradient of out is the next ResBlock's bn1-backward output; that pass writes
        # its e4m3 copy for this conv2's data gradient (`_fv_q8_consumer`, ResBlock2D.forward
        # tags out with it), and this block does the same for the block before it
        blk._fv_q8_consumer = (c2, fp8_site(c2, "dy", x.device)) if cs2.fp8 else None
        prev = getattr(x, "_fv_q8_consumer", None)
        ctx.q8_prev = prev if cs1.fp8 and xb is x else None
        ctx.blk, ctx.cs1, ctx.cs2, ctx.r1, ctx.r2, ctx.comm = blk, cs1, cs2, r1, r2, comm
        ctx.save_for_backward(x, xb, t1, a1, a2)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, xb, t1, a1, a2 = ctx.saved_tensors
        blk, cs1, cs2, r1, r2, comm = ctx.blk, ctx.cs1, ctx.cs2, ctx.r1, ctx.r2, ctx.comm
        C = xb.shape[1]
        dout = grad_in(dout, xb.dtype)
        # (the BN-backward sums stay a separate pass here: fused into the 256-channel dgrad's
        # store pass they cost that kernel +29 us per launch against the pass's 27 us,
        # profiles/r2b_*)
        # the e4m3 copy of dout, if the next block's bn1 backward wrote one for exactly this tensor
        # in exactly this state: the same tensor object at the same version.  A second consumer
        # of this block's output makes autograd add its gradient into that tensor in place (same
        # pointer, new version) or hand over a new tensor; either way the copy is stale and dout
        # is quantized again (the stale copy's amax already went into the site's in-flight slot:
        # an upper bound, only the next step's scale can be one power of two smaller than ideal)
        pend = cs2.conv.__dict__.pop("_fv_fp8_pending", None) if cs2.fp8 else None
        dy8 = None
        if pend is not None and _FP8_HANDOFF:
            t = pend[0]()
            if t is not None and t is dout and dout._version == pend[1]:
                dy8 = pend[2]
        # (the BN-backward sums reduced in the data gradients' store pass instead of the reduce
        # pass: step 12.46 -> 12.67 ms in r4, as in r2 -- DESIGN.md §4)
        da2, dw2, db2 = conv_backward(cs2, a2, dout, C, dy8=dy8)
        site1 = fp8_site(cs1.conv, "dy", xb.device) if cs1.fp8 else None
        dt1, dg2, dbe2, *q = bn_act_backward(da2, t1, blk.bn2, r2, 0.0, False, comm, q8=site1,
                                             only8=site1 is not None and q8_only(cs1))
        da1, dw1, db1 = conv_backward(cs1, a1, dt1, C, dy8=q[0] if q else None)
        prev = ctx.q8_prev
        dxb, dg1, dbe1, *q = bn_act_backward(da1, xb, blk.bn1, r1, 0.0, False, comm, addend=dout,
                                             q8=prev[1] if prev is not None else None)
        if prev is not None and q and q[0] is not None:
            prev[0].__dict__["_fv_fp8_pending"] = (weakref.ref(dxb), dxb._version, q[0])
        dx = from_nhwc(dxb, x)
        return dx, dw1, db1, dg1, dbe1, dw2, db2, dg2, dbe2, None


class NACFn(torch.autograd.Function):
    """Standalone "NAC" ConvBlock2D: conv(act(BN(x))), the BN-apply+act output materialised once."""

    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, blk):
        mode = blk.compute_dtype()
        dtype = storage(mode)
        xb, C = to_nhwc(x, dtype)
        if C != x.shape[1]:
            raise RuntimeError("NAC block input channels must be a power of two >= 8")
        N, _, H, W = x.shape
        conv = blk.conv
        cout = conv.out_channels
        if cout % 8:
            raise RuntimeError("NAC block output channels must be a multiple of 8")
        comm = blk.bn_comm()
        r = bn_from_tensor(blk.bn, xb, blk.training, comm)
        a = bn_act_forward(xb, r, blk.slope, False, blk.bn)
        d = desc(dtype, N, H, W, C, C, cout, cout, conv.kernel_size)
        cs = ConvState(conv, d, dtype, x.device, blk.training, need_wt=True, fp8=mode == FP8)
        y = torch.empty((N, cout, H, W), dtype=dtype, device=x.device, memory_format=CL)
        conv_forward(cs, a, bias, y=y)
        cs.release()
        ctx.blk, ctx.cs, ctx.r, ctx.comm = blk, cs, r, comm
        ctx.save_for_backward(x, xb, a)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, xb, a = ctx.saved_tensors
        blk, cs, r = ctx.blk, ctx.cs, ctx.r
        dy = grad_in(dy, xb.dtype)
        da, dw, db = conv_backward(cs, a, dy, dy.shape[1])
        dxb, dg, dbt = bn_act_backward(da, xb, blk.bn, r, blk.slope, False, ctx.comm,
                                       need_dx=ctx.needs_input_grad[0])
        return (from_nhwc(dxb, x) if dxb is not None else None), dw, db, dg, dbt, None


class ConvFn(torch.autograd.Function):
    """Plain nn.Conv2d (+ optional fused sigmoid with NCHW fp32 output: models.py:1099,1110)."""

    @staticmethod
    def forward(ctx, x, weight, bias, conv, mode, sigmoid):
        dtype = storage(mode)
        xb, cin_pad = to_nhwc(x, dtype)
        N, _, H, W = x.shape
        cout = conv.out_channels
        nchw = bool(sigmoid) or (cout % 8 != 0)
        d = desc(dtype, N, H, W, cin_pad, conv.in_channels, cout, cout, conv.kernel_size, sig=sigmoid, nchw=nchw)
        cs = ConvState(conv, d, dtype, x.device, conv.training, need_wt=ctx.needs_input_grad[0], fp8=mode == FP8)
        if nchw:
            y = torch.empty((N, cout, H, W), dtype=F32, device=x.device)
        else:
            y = torch.empty((N, cout, H, W), dtype=dtype, device=x.device, memory_format=CL)
        conv_forward(cs, xb, bias, y=y)
        cs.release()
        ctx.cs, ctx.sigmoid, ctx.nchw, ctx.dtype = cs, sigmoid, nchw, dtype
        ctx.save_for_backward(x, xb, y if sigmoid else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, xb, y = ctx.saved_tensors
        cs = ctx.cs
        d = cs.d
        dtype = ctx.dtype
        if ctx.nchw:
            ldd = pad_pow2(d.cout)
            dpre = torch.empty((d.n, ldd, d.h, d.w), dtype=dtype, device=dy.device, memory_format=CL)
            dy32 = dy.float().contiguous()
            if ctx.sigmoid:
                call("fv_sigmoid_bwd_to_nhwc", L.dtype_code(dtype), ptr(dy32), ptr(y), d.n, d.cout, d.h * d.w, ldd,
                     ptr(dpre), stream())
            else:
                call("fv_nchw_to_nhwc", L.dtype_code(dtype), ptr(dy32), d.n, d.cout, d.h * d.w, ldd, ptr(dpre),
                     stream())
        else:
            ldd = d.cout
            dpre = grad_in(dy, dtype)
        dxb, dw, db = conv_backward(cs, xb, dpre, ldd, need_dx=ctx.needs_input_grad[0])
        dx = from_nhwc(dxb, x) if dxb is not None else None
        return dx, dw, db, None, None, None


class ReparamFn(torch.autograd.Function):
    """mu = h[:, :L], logstd = h[:, L:], z = mu + exp(logstd) * eps (models.py:559-561).
    The same pass also reduces the KL of (mu, logstd) (losses.py:392); `reparameterise`
    tags mu with it so that KLDivergenceLoss on exactly this (mu, logstd) pair reuses the
    value instead of re-reading both tensors, and hands its gradient back through `holder`
    (`KLFn.backward`), which this backward folds into dh (fv_reparam_kl_bwd): no separate KL
    backward pass, no dmu / dlogstd tensors.  On the tiled shapes mu and logstd are the
    channel slices of the NHWC h itself (no copies written)."""

    @staticmethod
    def forward(ctx, h, eps, dtype, holder):
        ctx.set_materialize_grads(False)
        hb, C2 = to_nhwc(h, dtype)
        N, _, H, W = h.shape
        Lc = C2 // 2
        e32 = eps.float().contiguous()
        if tuple(e32.shape) != (N, Lc, H, W):
            raise RuntimeError(f"eps must be [N, {Lc}, {H}, {W}]")
        z = torch.empty((N, Lc, H, W), dtype=dtype, device=h.device, memory_format=CL)
        if query("fv_reparam_tiled", Lc, H * W):
            mu, ls = None, None
        else:
            mu, ls = torch.empty_like(z), torch.empty_like(z)
        kl = torch.empty((), dtype=F32, device=h.device)
        ws = _empty(query("fv_reparam_ws_bytes", N, Lc, H * W) // 8 + 1, F64, h.device)
        call("fv_reparam_kl_fwd", L.dtype_code(dtype), ptr(hb), ptr(e32), N, Lc, H * W, ptr(mu), ptr(ls), ptr(z),
             ptr(kl), ptr(ws), stream())
        if mu is None:
            mu, ls = hb[:, :Lc], hb[:, Lc:]
        holder["kl"] = kl
        ctx.save_for_backward(h, hb, e32)
        ctx.dtype = dtype
        ctx.holder = holder
        return mu, ls, z

    @staticmethod
    def backward(ctx, dmu, dls, dz):
        h, hb, e32 = ctx.saved_tensors
        N, C2, H, W = hb.shape
        dt = ctx.dtype
        klg = ctx.holder.pop("kl_grad", None)
        dh = torch.empty_like(hb, memory_format=CL)
        call("fv_reparam_kl_bwd", L.dtype_code(dt), ptr(hb), ptr(e32), N, C2 // 2, H * W,
             ptr(grad_in(dz, dt) if dz is not None else None),
             ptr(grad_in(dmu, dt) if dmu is not None else None),
             ptr(grad_in(dls, dt) if dls is not None else None), ptr(klg), ptr(dh), stream())
        return from_nhwc(dh, h), None, None, None


def _same_layout(a, b):
    if a.shape == b.shape and a.stride() == b.stride() and a.dtype == b.dtype and (
            a.is_contiguous() or nhwc_view(a)):
        return a, b
    return a.contiguous(), b.to(a.dtype).contiguous()


class KLFn(torch.autograd.Function):
    """mean(-0.5 - logstd + 0.5 mu^2 + 0.5 exp(2 logstd)) (losses.py:392)."""

    @staticmethod
    def forward(ctx, mu, logstd):
        pre = getattr(mu, "_fv_kl", None)
        ctx.holder = None
        if pre is not None and pre[0] is logstd and mu._version == pre[2] and logstd._version == pre[3]:
            ctx.holder = pre[4]                    # value reduced by the reparameterisation pass,
            return pre[1].clone()                  # gradient folded into its backward
        if mu.dtype not in (F32, torch.bfloat16):
            mu, logstd = mu.float(), logstd.float()
        mu, logstd = _same_layout(mu, logstd)
        out = torch.empty((), dtype=F32, device=mu.device)
        ws = _empty(query("fv_loss_ws_bytes") // 8, F64, mu.device)
        call("fv_kl_fwd", L.dtype_code(mu.dtype), ptr(mu), ptr(logstd), mu.numel(), ptr(out), ptr(ws), stream())
        ctx.save_for_backward(mu, logstd)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.float().reshape(())
        if ctx.holder is not None:
            prev = ctx.holder.get("kl_grad")
            ctx.holder["kl_grad"] = g.contiguous() if prev is None else prev + g
            return None, None
        mu, ls = ctx.saved_tensors
        dmu = torch.empty_like(mu) if ctx.needs_input_grad[0] else None
        dls = torch.empty_like(ls) if ctx.needs_input_grad[1] else None
        call("fv_kl_bwd", L.dtype_code(mu.dtype), ptr(mu), ptr(ls), mu.numel(), ptr(g), ptr(dmu), ptr(dls), stream())
        return dmu, dls


class _PairLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, kind):
        a32 = a.float()
        b32 = b.float()
        a32, b32 = _same_layout(a32, b32)
        out = torch.empty((), dtype=F32, device=a.device)
        ws = _empty(query("fv_loss_ws_bytes") // 8, F64, a.device)
        call("fv_mse_fwd" if kind == "mse" else "fv_l1_fwd", ptr(a32), ptr(b32), a32.numel(), ptr(out), ptr(ws),
             stream())
        ctx.save_for_backward(a32, b32)
        ctx.kind = kind
        ctx.dt = (a.dtype, b.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.float().contiguous()
        da = torch.empty_like(a) if ctx.needs_input_grad[0] else None
        db = torch.empty_like(b) if ctx.needs_input_grad[1] else None
        call("fv_mse_bwd" if ctx.kind == "mse" else "fv_l1_bwd", ptr(a), ptr(b), a.numel(), ptr(g), ptr(da),
             ptr(db), stream())
        return (da.to(ctx.dt[0]) if da is not None else None, db.to(ctx.dt[1]) if db is not None else None, None)


def mse_loss(a, b):
    return _PairLossFn.apply(a, b, "mse")


def l1_loss(a, b):
    return _PairLossFn.apply(a, b, "l1")


def kl_loss(mu, logstd):
    return KLFn.apply(mu, logstd)


def reparameterise(h, eps, mode):
    dtype = storage(mode)
    holder = {}
    mu, ls, z = ReparamFn.apply(h, eps, dtype, holder)
    mu._fv_kl = (ls, holder["kl"], mu._version, ls._version, holder)
    return mu, ls, z


class ConvTranspose2dFn(torch.autograd.Function):
    """F.conv_transpose2d(x, gain * [demod-normalised] W, stride=2, padding=1) + bias with a
    4x4 kernel (ConvTranspose2dELR.getweight/forward, models_utils.py:454-505), on the
    sub-pixel upsample-conv kernels (include/facevae.h, "transposed conv").  bf16 only."""

    @staticmethod
    def forward(ctx, x, weight, bias, demod, gain):
        dtype = torch.bfloat16
        xb, cin_pad = to_nhwc(x, dtype)
        N, inch, Hi, Wi = x.shape
        outch = weight.shape[1]
        if weight.dtype != F32 or not weight.is_contiguous():
            raise RuntimeError("conv_transpose2d weights must be contiguous fp32")
        d = desc(dtype, N, 2 * Hi, 2 * Wi, cin_pad, inch, outch, outch, 3, ups=1)
        if not query("fv_convt_supported", ctypes.byref(d)):
            raise RuntimeError(f"conv_transpose2d (k4 s2 p1): unsupported shape in={tuple(x.shape)} outch={outch} "
                               "(needs inch > 32, outch a power of two >= 64, input height and width powers of two, width >= 64)")
        dev = x.device
        inv = torch.empty(outch, dtype=F32, device=dev)
        wk = _empty(query("fv_conv_wk_elems", ctypes.byref(d)), dtype, dev)
        wt = _empty(query("fv_conv_wt_elems", ctypes.byref(d)), dtype, dev) if ctx.needs_input_grad[0] else None
        call("fv_convt_weight_prep", ctypes.byref(d), ptr(weight), int(demod), float(gain), ptr(inv), ptr(wk),
             ptr(wt), stream())
        y = torch.empty((N, outch, 2 * Hi, 2 * Wi), dtype=dtype, device=dev, memory_format=CL)
        call("fv_conv2d_fwd", ctypes.byref(d), ptr(xb), ptr(wk), ptr(bias), None, None, None, ptr(y), None, stream())
        ctx.d, ctx.demod, ctx.gain, ctx.wt, ctx.has_bias = d, int(demod), float(gain), wt, bias is not None
        ctx.save_for_backward(x, xb, weight, inv)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, xb, weight, inv = ctx.saved_tensors
        d = ctx.d
        dev = dy.device
        dy = grad_in(dy, torch.bfloat16)
        slab = _empty(query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), F32, dev)
        bslab = _empty(query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), F32, dev)
        call("fv_conv2d_bwd_weight", ctypes.byref(d), ptr(xb), None, None, ptr(dy), d.cout, ptr(slab), ptr(bslab),
             stream())
        dw = torch.empty_like(weight)
        db = torch.empty(d.cout, dtype=F32, device=dev) if ctx.has_bias else None
        call("fv_convt_wgrad_reduce", ctypes.byref(d), ptr(slab), ptr(bslab), ptr(weight), ctx.demod, ctx.gain,
             ptr(inv), ptr(dw), ptr(db), stream())
        dx = None
        if ctx.needs_input_grad[0]:
            dxb = torch.empty((d.n, d.cin, d.h // 2, d.w // 2), dtype=dy.dtype, device=dev, memory_format=CL)
            call("fv_conv2d_bwd_data", ctypes.byref(d), ptr(dy), d.cout, ptr(ctx.wt), ptr(dxb), stream())
            dx = from_nhwc(dxb, x)
        return dx, dw, db, None, None


class ConvTranspose2dDirectFn(torch.autograd.Function):
    """F.conv_transpose2d(x, gain * [demod-normalised] W, stride, padding) + bias for any
    geometry and for fp32 parity mode (ConvTranspose2dELR.getweight/forward,
    models_utils.py:454-505) on the direct kernels of convt.hip."""

    @staticmethod
    def forward(ctx, x, weight, bias, k, stride, pad, demod, gain, dtype):
        xb, ldx = to_nhwc(x, dtype)
        N, inch, Hi, Wi = x.shape
        outch = weight.shape[1]
        if weight.dtype != F32 or not weight.is_contiguous():
            raise RuntimeError("conv_transpose2d weights must be contiguous fp32")
        Ho, Wo = (Hi - 1) * stride - 2 * pad + k, (Wi - 1) * stride - 2 * pad + k
        dev = x.device
        inv = torch.empty(outch, dtype=F32, device=dev)
        we = torch.empty_like(weight)
        call("fv_convt_eff_weight", ptr(weight), inch, outch, k, int(demod), float(gain), ptr(inv), ptr(we), stream())
        y = torch.empty((N, outch, Ho, Wo), dtype=dtype, device=dev, memory_format=CL)
        call("fv_convt_direct_fwd", L.dtype_code(dtype), ptr(xb), N, Hi, Wi, inch, ldx, ptr(we), ptr(bias), outch, outch,
             k, stride, pad, ptr(y), stream())
        ctx.geo = (k, stride, pad, int(demod), float(gain), ldx)
        ctx.dtype, ctx.has_bias = dtype, bias is not None
        ctx.save_for_backward(x, xb, weight, we, inv)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, xb, weight, we, inv = ctx.saved_tensors
        k, stride, pad, demod, gain, ldx = ctx.geo
        N, inch, Hi, Wi = x.shape
        outch = weight.shape[1]
        dyb = dy.to(ctx.dtype).contiguous(memory_format=CL)
        g = torch.empty_like(weight)
        db = torch.empty(outch, dtype=F32, device=dy.device) if ctx.has_bias else None
        call("fv_convt_direct_wgrad", L.dtype_code(ctx.dtype), ptr(xb), ptr(dyb), N, Hi, Wi, inch, ldx, outch, outch, k,
             stride, pad, ptr(g), ptr(db), stream())
        call("fv_convt_weight_grad", ptr(weight), inch, outch, k, demod, gain, ptr(inv), ptr(g), stream())
        dx = None
        if ctx.needs_input_grad[0]:
            dxb = torch.empty((N, ldx, Hi, Wi), dtype=ctx.dtype, device=dy.device, memory_format=CL)
            call("fv_convt_direct_dgrad", L.dtype_code(ctx.dtype), ptr(dyb), N, Hi, Wi, inch, ldx, ptr(we), outch, outch,
                 k, stride, pad, ptr(dxb), stream())
            dx = from_nhwc(dxb, x)
        return dx, g, db, None, None, None, None, None, None


class ChanScaleFn(torch.autograd.Function):
    """y[n, c] = x[n, c] * sa[n, c] (+ sb[n, c]) over an NHWC activation (the per-sample
    modulation / demodulation of ConvTranspose2dELR, models_utils.py:486-495)."""

    @staticmethod
    def forward(ctx, x, sa, sb, dtype):
        xb, ld = to_nhwc(x, dtype)
        N, C, H, W = x.shape
        sa32 = sa.float().contiguous()
        sb32 = sb.float().contiguous() if sb is not None else None
        y = torch.empty((N, ld, H, W), dtype=dtype, device=x.device, memory_format=CL).zero_() if ld != C else torch.empty_like(xb)
        call("fv_chan_scale_fwd", L.dtype_code(dtype), ptr(xb), N, H * W, C, ld, ptr(sa32), ptr(sb32), ptr(y), stream())
        ctx.save_for_backward(x, xb, sa32)
        ctx.dtype, ctx.has_sb = dtype, sb is not None
        return y if ld == C else from_nhwc(y, x.to(dtype))

    @staticmethod
    def backward(ctx, g):
        x, xb, sa32 = ctx.saved_tensors
        N, C, H, W = x.shape
        gb, ld = to_nhwc(g, ctx.dtype)
        dx = torch.zeros_like(xb) if ctx.needs_input_grad[0] else None
        da = torch.empty((N, C), dtype=F32, device=g.device)
        db = torch.empty((N, C), dtype=F32, device=g.device) if ctx.has_sb else None
        call("fv_chan_scale_bwd", L.dtype_code(ctx.dtype), ptr(gb), ptr(xb), N, H * W, C, ld, ptr(sa32), ptr(dx),
             ptr(da), ptr(db), stream())
        return (from_nhwc(dx, x) if dx is not None else None), da, db, None
