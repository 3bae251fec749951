"""Torch fp32 references of the conv launches of the model path, for the per-launch parity
checks (ops.CHECK hook).  Test infrastructure only.

Each reference takes the SAME operands the HIP kernel consumed (the bf16 activation / gradient
tensors as stored in HBM, the weights rounded to the compute dtype exactly as
fv_conv_weight_prep rounds them) and computes the op in fp32 on the GPU with explicit
im2col (F.unfold / F.fold) + GEMM — no MIOpen, no TF32 — chunked over the batch so the column
matrices stay a few GB.  What remains between kernel and reference is then only the kernel's
own error: fp32 summation order and the final rounding of a bf16 output.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False

_CHUNK_BYTES = 3 << 30


def _nb(n, per_image_bytes):
    return max(1, min(n, _CHUNK_BYTES // max(1, per_image_bytes)))


def eff_weight(cs, dtype) -> torch.Tensor:
    """[co][ci][k][k] fp32 weight the kernel multiplies by: (w / sigma) rounded to `dtype`."""
    w = cs.w.detach()
    if cs.sigma is not None:
        w = w * (1.0 / cs.sigma.detach().float())
    return w.to(dtype).float()


def pro_input(x, pro, slope, dtype):
    """act(x * scale + shift) per channel, rounded to the compute dtype (the kernel stages the
    transformed bf16 operand)."""
    if pro is None:
        return x
    sc, sh = pro
    v = x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
    v = torch.where(v > 0, v, v * slope)
    return v.to(dtype).float()


def conv_fwd_ref(x, w, bias, k, ups):
    if ups:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    N, C, H, W = x.shape
    co = w.shape[0]
    wm = w.reshape(co, -1)
    out = torch.empty(N, co, H, W, device=x.device, dtype=torch.float32)
    nb = _nb(N, C * k * k * H * W * 4)
    for n0 in range(0, N, nb):
        cols = F.unfold(x[n0:n0 + nb], k, padding=k // 2)
        out[n0:n0 + nb] = (wm @ cols).view(-1, co, H, W)
    if bias is not None:
        out += bias.view(1, -1, 1, 1)
    return out


def _fold_rows(p, r_):
    """3x3 taps r folded into 2x2 tap r_ of sub-pixel phase p (weight_prep_subpix_kernel)."""
    return range(1 + p, 3) if r_ else range(0, p + 1)


def subpix_fwd_ref(x, w, bias, dtype):
    """nearest-x2 + 3x3 conv as the kernel computes it: 4 sub-pixel phases of a 2x2 conv over
    the low-res input with phase-folded weights (summed in fp32, then rounded to `dtype`)."""
    N, C, H, W = x.shape
    co = w.shape[0]
    out = torch.empty(N, co, 2 * H, 2 * W, device=x.device, dtype=torch.float32)
    for pa in range(2):
        for pb in range(2):
            wp = torch.zeros(co, C, 2, 2, device=w.device, dtype=torch.float32)
            for r_ in range(2):
                for s_ in range(2):
                    for r in _fold_rows(pa, r_):
                        for q in _fold_rows(pb, s_):
                            wp[:, :, r_, s_] += w[:, :, r, q]
            wm = wp.to(dtype).float().reshape(co, -1)
            xp = F.pad(x, (1 - pb, pb, 1 - pa, pa))
            nb = _nb(N, C * 4 * H * W * 4)
            for n0 in range(0, N, nb):
                cols = F.unfold(xp[n0:n0 + nb], 2)
                out[n0:n0 + nb, :, pa::2, pb::2] = (wm @ cols).view(-1, co, H, W)
    if bias is not None:
        out += bias.view(1, -1, 1, 1)
    return out


def lowres_dgrad_ref(dy, w, dtype):
    """Data gradient of nearest-x2 + 3x3 straight at the low resolution, as the kernel
    computes it: a stride-2 4x4 conv over dy with tap-folded weights rounded to `dtype`
    (weight_prep_s2_kernel)."""
    N, co, H, W = dy.shape
    ci = w.shape[1]
    wt = torch.zeros(ci, co, 4, 4, device=w.device, dtype=torch.float32)
    for tr in range(4):
        for tc in range(4):
            for r in range(max(0, 2 - tr), min(2, 3 - tr) + 1):
                for q in range(max(0, 2 - tc), min(2, 3 - tc) + 1):
                    wt[:, :, tr, tc] += w[:, :, r, q].t()
    wm = wt.to(dtype).float().reshape(ci, -1)
    dx = torch.empty(N, ci, H // 2, W // 2, device=dy.device, dtype=torch.float32)
    nb = _nb(N, co * 16 * H * W)
    for n0 in range(0, N, nb):
        cols = F.unfold(dy[n0:n0 + nb], 4, padding=1, stride=2)
        dx[n0:n0 + nb] = (wm @ cols).view(-1, ci, H // 2, W // 2)
    return dx


def conv_dgrad_ref(dy, w, k, ups, in_hw):
    """Gradient w.r.t. the conv input (at the upsampled resolution when ups, then summed back
    over each 2x2 block = nearest-upsample backward)."""
    N, co, H, W = dy.shape
    ci = w.shape[1]
    wt = w.reshape(co, -1).t()
    dx = torch.empty(N, ci, H, W, device=dy.device, dtype=torch.float32)
    nb = _nb(N, ci * k * k * H * W * 4)
    for n0 in range(0, N, nb):
        cols = wt @ dy[n0:n0 + nb].reshape(-1, co, H * W)
        dx[n0:n0 + nb] = F.fold(cols, (H, W), k, padding=k // 2)
    if ups:
        dx = F.avg_pool2d(dx, 2) * 4
    return dx


def conv_wgrad_ref(x, dy, k, ups):
    if ups:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    N, C, H, W = x.shape
    co = dy.shape[1]
    acc = torch.zeros(co, C * k * k, device=x.device, dtype=torch.float64)
    nb = _nb(N, C * k * k * H * W * 8)
    for n0 in range(0, N, nb):                                        # fp64: exact for bf16 operands
        cols = F.unfold(x[n0:n0 + nb].double(), k, padding=k // 2)   # [nb, C k k, HW]
        d = dy[n0:n0 + nb].double().reshape(-1, co, H * W)
        acc += torch.einsum("npk,nqk->pq", d, cols)
    return acc.view(co, C, k, k), dy.double().sum((0, 2, 3))


def compare_sum(out, ref, ref_abs, unit=2.0 ** -14):
    """fp32 results of long reductions (weight / bias gradients: sums over every pixel of the
    batch, reference in fp64): elementwise bound 2^-14 of the sum of |terms| -- a block's fp32
    accumulators run sequentially over up to ~16k pixels of its split, sqrt(16k) * 2^-24 ~
    2^-17 typical -- with the global rel-L2 (gated at 1e-4 for weight gradients) catching a
    missing or doubled split.  unit: the bound's multiple of sum|terms| (2^-10 for the fp8 weight
    gradient: the scaled fp8 MFMA adds its products in groups of 8 truncated ~13 bits below the
    group's largest, tests/test_fp8_gpu.py::test_fp8_mfma_accumulation_groups)."""
    d = (out.double() - ref).abs()
    rl2 = (d.norm() / ref.norm().clamp_min(1e-30)).item()
    worst = (d / (unit * ref_abs + 1e-30)).max().item()
    return rl2, worst


def compare(out, ref, aux=None, out_bf16=True):
    """(rel-L2, worst elementwise ratio |d| / bound).  bound = rounding of a bf16 output
    (2^-7 of the value, plus the residual it was added to) + 2e-3 of the reference's RMS for
    fp32 summation-order noise; for fp32 outputs (weight gradients, the fp32 image) 1e-4 of the
    value + 1e-4 of the RMS.  A localised fault (a bad tile, a mis-staged halo row) shows up
    as a ratio >> 1 even when the global rel-L2 barely moves."""
    out = out.float()
    d = (out - ref).abs()
    rms = ref.pow(2).mean().sqrt().clamp_min(1e-30)
    if out_bf16:
        bound = 2.0 ** -7 * (ref.abs() + (aux.float().abs() if aux is not None else 0)) + 2e-3 * rms
    else:
        bound = 1e-4 * ref.abs() + 1e-4 * rms
    rl2 = (d.norm() / ref.norm().clamp_min(1e-30)).item()
    worst = (d / bound).max().item()
    return rl2, worst


class LaunchChecker:
    """ops.CHECK implementation: runs the reference of every conv launch right after it and
    records {layer, kind, shape, rel-L2, worst ratio}."""

    def __init__(self, model, dtype):
        from facevae_amd import _lib as L
        import ctypes
        self.dtype = torch.bfloat16 if dtype == torch.float8_e4m3fn else dtype
        # which formulation the library runs for an upsample conv (the sub-pixel phases have a
        # 4 x [rows][Kpad(2x2)] weight buffer; the low-res data gradient is reported directly)
        def subpix(d):
            bn = 128 if d.cout > 64 else 64 if d.cout > 32 else 32 if d.cout > 16 else 16   # conv.hip fwd_tile
            rows = (d.cout + bn - 1) // bn * bn
            return L.query("fv_conv_wk_elems", ctypes.byref(d)) == 4 * rows * ((4 * d.cin + 31) // 32 * 32)
        self.subpix = subpix
        self.lowres = lambda d: bool(L.query("fv_conv2d_dgrad_lowres", ctypes.byref(d)))
        self.names = {id(m): n for n, m in model.named_modules()}
        self.rows: List[Dict] = []

    def bn_fwd(self, bn, t):
        y = t["y"].float()
        r = t["r"]
        z = y * r.scale.view(1, -1, 1, 1) + r.shift.view(1, -1, 1, 1)
        z = torch.where(z > 0, z, z * t["slope"])
        if t["pool"]:
            z = F.avg_pool2d(z, 2)
        name = self.names.get(id(bn), "?")
        rl2, worst = compare(t["out"], z, out_bf16=self.dtype == torch.bfloat16)
        self._addbn(name, "bn_fwd", y.shape, rl2, worst)
        self.bn_stat(bn, t)

    def bn_stat(self, bn, t):
        """Batch statistics of a training-mode BN."""
        r = t["r"]
        name = self.names.get(id(bn), "?")
        if r.count or r.stats is not None:              # training: batch statistics
            y = t["y"]
            yd = t["y"].double()
            m = yd.mean((0, 2, 3))
            sd = yd.var((0, 2, 3), unbiased=False).add(bn.eps).sqrt()
            em = ((r.mean.double() - m).abs() / sd).max().item()
            ei = (r.invstd.double() * sd - 1).abs().max().item()
            self._addbn(name, "bn_stat", y.shape, max(em, ei), max(em, ei) / 2e-3)

    def bn_bwd(self, bn, t):
        y = t["y"].double()
        r = t["r"]
        mean, inv = r.mean.double().view(1, -1, 1, 1), r.invstd.double().view(1, -1, 1, 1)
        gam, bet = bn.weight.detach().double().view(1, -1, 1, 1), bn.bias.detach().double().view(1, -1, 1, 1)
        yh = (y - mean) * inv
        # the activation mask exactly as the kernel forms it (fp32), plus the elements whose
        # pre-activation sits within rounding of 0 (either side is then correct)
        yh32 = (t["y"].float() - r.mean.view(1, -1, 1, 1)) * r.invstd.view(1, -1, 1, 1)
        z32 = bn.weight.detach().view(1, -1, 1, 1) * yh32 + bn.bias.detach().view(1, -1, 1, 1)
        amb = z32.abs() <= 1e-5 * (bn.bias.detach().abs().view(1, -1, 1, 1) + (bn.weight.detach().view(1, -1, 1, 1) * yh32).abs())
        d = t["dout"].double()
        if t["pool"]:
            d = d.repeat_interleave(2, 2).repeat_interleave(2, 3) * 0.25
        g = d * torch.where(z32 > 0, 1.0, float(t["slope"])).double()
        dbeta, dgamma = g.sum((0, 2, 3)), (g * yh).sum((0, 2, 3))
        name = self.names.get(id(bn), "?")
        self._addbn(name, "dbeta", y.shape, *compare_sum(t["dbt"], dbeta, g.abs().sum((0, 2, 3))))
        self._addbn(name, "dgamma", y.shape, *compare_sum(t["dg"], dgamma, (g * yh).abs().sum((0, 2, 3))))
        if t["dx"] is not None:
            if r.count or r.stats is not None:
                n = y.shape[0] * y.shape[2] * y.shape[3]
                dx = gam * inv * (g - dbeta.view(1, -1, 1, 1) / n - yh * (dgamma.view(1, -1, 1, 1) / n))
            else:
                dx = gam * inv * g
            aux = None
            if t["addend"] is not None:
                aux = t["addend"].float()
                dx = dx + aux.double()
            ok = ~amb
            out = t["dx"].float()[ok]
            rl2, worst = compare(out, dx.float()[ok], aux[ok] if aux is not None else None,
                                 out_bf16=self.dtype == torch.bfloat16)
            self._addbn(name, "bn_dx", y.shape, rl2, worst)

    def _addbn(self, name, kind, shape, rl2, worst):
        self.rows.append({"layer": name, "kind": kind, "n": shape[0], "hw": (shape[2], shape[3]), "cin": shape[1],
                          "cout": shape[1], "k": 0, "ups": 0, "rel_l2": rl2, "worst": worst})

    def __call__(self, kind, cs, **t):
        if kind in ("bn_fwd", "bn_bwd", "bn_stat"):
            with torch.no_grad():
                return {"bn_fwd": self.bn_fwd, "bn_bwd": self.bn_bwd, "bn_stat": self.bn_stat}[kind](cs, t)
        d = cs.d
        name = self.names.get(id(cs.conv), "?")
        k = d.ksize
        ups = bool(d.upsample)
        w = eff_weight(cs, self.dtype)
        bf = self.dtype == torch.bfloat16
        with torch.no_grad():
            if kind in ("fwd", "dgrad") and t.get("q8") is not None:
                # the e4m3 operand (quantized by the conv's own pass, or written by its producer:
                # a BN pass, the next ResBlock's bn1 backward) is exactly its bf16 tensor x the
                # delayed scale, saturated
                q8, dq = t["q8"]
                src = t["x"] if kind == "fwd" else t["dy"]
                ref8 = (src.float() * (1.0 / dq.item())).clamp(-448, 448).to(torch.float8_e4m3fn)
                ref8 = ref8.permute(0, 2, 3, 1).reshape(-1).view(torch.uint8)
                bad = int((q8.reshape(-1) != ref8).sum().item())
                assert bad == 0, f"{name} {kind}: fp8 operand differs from its bf16 tensor in {bad} bytes"
            if kind == "fwd" and t.get("q8") is not None:        # fp8 kernel: dequantized operands
                x8, xdq = t["q8"]
                N, Cp, H, W = t["x"].shape
                xq = x8.view(torch.float8_e4m3fn).float().view(N, H, W, Cp).permute(0, 3, 1, 2) * xdq
                wq = cs.wk.view(torch.float8_e4m3fn).float().view(d.cout, 3, 3, d.cin).permute(0, 3, 1, 2) * cs.wdq
                ref = conv_fwd_ref(xq.contiguous(), wq.contiguous(), t["bias"], 3, False)
                aux = None
                if t.get("res") is not None:
                    aux = t["res"][:, :d.cout].float()
                    ref = ref + aux
                rl2, worst = compare(t["y"][:, :d.cout].float(), ref, aux, out_bf16=True)
                self._add(name, "fwd8", d, rl2, worst)
            elif kind == "dgrad" and t.get("q8") is not None:
                dy8, dydq = t["q8"]
                N, Co, H, W = t["dy"].shape
                dyq = dy8.view(torch.float8_e4m3fn).float().view(N, H, W, Co).permute(0, 3, 1, 2) * dydq
                wtq = cs.wt.view(torch.float8_e4m3fn).float().view(d.cin, 3, 3, d.cout).permute(0, 3, 1, 2) * cs.wdq
                ref = conv_fwd_ref(dyq.contiguous(), wtq.contiguous(), None, 3, False)
                rl2, worst = compare(t["dx"].float(), ref, out_bf16=True)
                self._add(name, "dgrad8", d, rl2, worst)
            elif kind == "fwd":
                x = t["x"][:, :d.cin_valid].float()
                x = pro_input(x, t.get("pro"), d.pro_slope, self.dtype)
                if ups and self.subpix(d):
                    ref = subpix_fwd_ref(x, eff_weight(cs, torch.float32), t["bias"], self.dtype)
                else:
                    ref = conv_fwd_ref(x, w, t["bias"], k, ups)
                y = t["y"]
                aux = None
                if t.get("res") is not None:
                    aux = t["res"][:, :d.cout].float()
                    ref = ref + aux
                if d.epi_sigmoid:
                    ref = torch.sigmoid(ref)
                y = y[:, :d.cout].float()
                rl2, worst = compare(y, ref, aux, out_bf16=bf and not d.out_nchw_f32)
                self._add(name, kind, d, rl2, worst)
            elif kind == "dgrad":
                dy = t["dy"][:, :d.cout].float()
                if ups and self.lowres(d):
                    ref = lowres_dgrad_ref(dy, eff_weight(cs, torch.float32), self.dtype)
                else:
                    ref = conv_dgrad_ref(dy, w, k, ups, None)
                dx = t["dx"][:, :d.cin_valid].float()
                rl2, worst = compare(dx, ref[:, :d.cin_valid], out_bf16=bf)
                self._add(name, kind, d, rl2, worst)
            elif t.get("q8") is not None:                 # fp8 weight gradient: dequantized operands
                x8, xdq, dy8, dydq = t["q8"]
                N, Cp, H, W = t["x"].shape
                xq = x8.view(torch.float8_e4m3fn).float().view(N, H, W, Cp).permute(0, 3, 1, 2) * xdq
                dyq = dy8.view(torch.float8_e4m3fn).float().view(N, H, W, d.cout).permute(0, 3, 1, 2) * dydq
                rw, rb = conv_wgrad_ref(xq.contiguous(), dyq.contiguous(), k, ups)
                aw, ab = conv_wgrad_ref(xq.abs().contiguous(), dyq.abs().contiguous(), k, ups)
                rl2, worst = compare_sum(t["dw"], rw, aw, unit=2.0 ** -10)
                self._add(name, "wgrad8", d, rl2, worst)
                if t.get("db") is not None:
                    rl2b, wb = compare_sum(t["db"], rb, ab, unit=2.0 ** -10)
                    self._add(name, "bgrad8", d, rl2b, wb)
            else:
                x = t["x"][:, :d.cin_valid].float()
                x = pro_input(x, t.get("pro"), d.pro_slope, self.dtype)
                dy = t["dy"][:, :d.cout].float()
                rw, rb = conv_wgrad_ref(x, dy, k, ups)
                aw, ab = conv_wgrad_ref(x.abs(), dy.abs(), k, ups)
                rl2, worst = compare_sum(t["dw"], rw, aw)
                self._add(name, kind, d, rl2, worst)
                if t.get("db") is not None:
                    rl2b, wb = compare_sum(t["db"], rb, ab)
                    self._add(name, "bgrad", d, rl2b, wb)

    def _add(self, name, kind, d, rl2, worst):
        self.rows.append({"layer": name, "kind": kind, "n": d.n, "hw": (d.h, d.w), "cin": d.cin_valid,
                          "cout": d.cout, "k": d.ksize, "ups": d.upsample, "rel_l2": rl2, "worst": worst})

    def report(self):
        lines = [f"{'layer':44s} {'kind':6s} {'shape':28s} {'rel-L2':>9s} {'worst':>7s}"]
        for r in self.rows:
            shp = f"n{r['n']} {r['hw'][0]}x{r['hw'][1]} {r['cin']}->{r['cout']} k{r['k']}{' up' if r['ups'] else ''}"
            lines.append(f"{r['layer']:44s} {r['kind']:6s} {shp:28s} {r['rel_l2']:9.2e} {r['worst']:7.3f}")
        return "\n".join(lines)
