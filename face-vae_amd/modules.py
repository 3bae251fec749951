"""Drop-in building blocks with the reference constructor signatures and state-dict keys
(modules.py:8-130 of Luh1124/face-vae), computed by the HIP kernels in ops.py.

Parameter / buffer layout is identical to the reference (e.g. `layers.0.weight_orig`,
`layers.0.weight_u`, `layers.1.running_mean`), and construction draws the same RNG
sequence as the reference constructors (nn.Conv2d.reset_parameters, then spectral_norm's
u/v), so `torch.manual_seed(s)` gives bit-identical initial weights.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn.functional as F
from torch import nn

from . import config
from . import ops


class _Conv(nn.Module):
    """Parameter holder of one conv: `weight` + `bias` or, with spectral norm,
    `bias` + `weight_orig` + buffers `weight_u`/`weight_v` (torch/nn/utils/spectral_norm.py:163-181)."""

    def __init__(self, in_channels, out_channels, kernel_size, use_sn=False, bias=True):
        super().__init__()
        self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, kernel_size
        self.sn = use_sn
        w = torch.empty(out_channels, in_channels, kernel_size, kernel_size)
        b = torch.empty(out_channels) if bias else None
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))           # nn.Conv2d.reset_parameters
        if b is not None:
            bound = 1.0 / math.sqrt(in_channels * kernel_size * kernel_size)
            nn.init.uniform_(b, -bound, bound)
        if use_sn:
            with torch.no_grad():
                u = F.normalize(w.new_empty(out_channels).normal_(0, 1), dim=0, eps=1e-12)
                v = F.normalize(w.new_empty(w[0].numel()).normal_(0, 1), dim=0, eps=1e-12)
            self.bias = nn.Parameter(b) if b is not None else None
            self.weight_orig = nn.Parameter(w)
            self.register_buffer("weight_u", u)
            self.register_buffer("weight_v", v)
        else:
            self.weight = nn.Parameter(w)
            self.bias = nn.Parameter(b) if b is not None else None

    def weight_param(self):
        return self.weight_orig if self.sn else self.weight

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, sn={self.sn}"


class _BatchNorm(nn.Module):
    """SyncBatchNorm parameter/buffer holder (modules.py:19); statistics are synchronised
    across ranks when a communicator is installed (distributed.py)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.track_running_stats = True
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def extra_repr(self):
        return f"{self.num_features}, eps={self.eps}, momentum={self.momentum}"


class _Act(nn.Module):
    def __init__(self, kind):
        super().__init__()
        self.kind = kind
        self.slope = 0.0 if kind == "relu" else 0.2

    def extra_repr(self):
        return self.kind


class _Upsample(nn.Module):
    def extra_repr(self):
        return "scale_factor=2, mode=nearest (folded into the conv addressing)"


class _AvgPool(nn.Module):
    def extra_repr(self):
        return "kernel_size=2 (fused into the BN/act pass)"


def _ref(owner, name, module):
    """Keep a plain (unregistered) reference to a submodule: no duplicate state-dict keys."""
    object.__setattr__(owner, name, module)


class _Block(nn.Module):
    """Common plumbing: compute dtype and the SyncBN communicator."""

    _dtype = None

    def compute_dtype(self):
        return self._dtype or config.compute_dtype()

    def set_compute_dtype(self, dtype):
        for m in self.modules():
            if hasattr(m, "_dtype"):
                m._dtype = dtype
        return self

    def bn_comm(self):
        from . import distributed
        return distributed.syncbn_comm() if self.training else None


class ConvBlock2D(_Block):
    """_ConvBlock (modules.py:8-49).  Patterns "CNA" (BN on the output) and "NAC" (BN on the
    input) are fused into one kernel chain; stride must be 1 and padding kernel_size // 2."""

    def __init__(self, pattern, in_channels, out_channels, kernel_size, stride, padding, use_weight_norm,
                 activation_type="batch", nonlinearity_type="relu"):
        super().__init__()
        if stride != 1 or padding != kernel_size // 2:
            raise NotImplementedError("facevae_amd ConvBlock2D: stride 1, 'same' padding only")
        if activation_type != "batch":
            raise NotImplementedError("facevae_amd ConvBlock2D: activation_type='batch' only")
        if pattern not in ("CNA", "NAC"):
            raise NotImplementedError(f"pattern {pattern}")
        self.pattern = pattern
        norm_channels = out_channels if pattern.find("C") < pattern.find("N") else in_channels
        mappings = {"C": _Conv(in_channels, out_channels, kernel_size, use_weight_norm),
                    "N": _BatchNorm(norm_channels),
                    "A": _Act(nonlinearity_type)}
        self.layers = nn.Sequential(*[mappings[c] for c in pattern])
        _ref(self, "conv", mappings["C"])
        _ref(self, "bn", mappings["N"])
        _ref(self, "act", mappings["A"])
        self.slope = self.act.slope
        self.upsample = False
        self.pool = False

    def forward(self, x):
        if self.pattern == "CNA":
            z = ops.ConvBNActFn.apply(x, self.conv.weight_param(), self.conv.bias, self.bn.weight, self.bn.bias, self)
            holder = getattr(self, "_fv_holder", None)
            if holder is not None and z.requires_grad:
                z._fv_bnsrc = (holder, z._version)   # read by the consuming conv (ops._claim_bnsrc)
            return z
        return ops.NACFn.apply(x, self.conv.weight_param(), self.conv.bias, self.bn.weight, self.bn.bias, self)


class DownBlock2D(_Block):
    """CNA 3x3 then AvgPool2d(2) (modules.py:59-70); pool fused into the BN/act pass."""

    def __init__(self, in_channels, out_channels, use_weight_norm):
        super().__init__()
        cb = ConvBlock2D("CNA", in_channels, out_channels, 3, 1, 1, use_weight_norm)
        cb.pool = True
        self.layers = nn.Sequential(cb, _AvgPool())

    def forward(self, x):
        return self.layers[0](x)


class UpBlock2D(_Block):
    """Upsample(x2, nearest) then CNA 3x3 (modules.py:78-89); the upsample is folded into the
    conv's input addressing, never materialised."""

    def __init__(self, in_channels, out_channels, use_weight_norm):
        super().__init__()
        cb = ConvBlock2D("CNA", in_channels, out_channels, 3, 1, 1, use_weight_norm)
        cb.upsample = True
        self.layers = nn.Sequential(_Upsample(), cb)

    def forward(self, x):
        return self.layers[1](x)


class SameBlock2D(_Block):
    """CNA 1x1 (modules.py:97-108)."""

    def __init__(self, in_channels, out_channels, use_weight_norm):
        super().__init__()
        self.layers = ConvBlock2D("CNA", in_channels, out_channels, 1, 1, 0, use_weight_norm)

    def forward(self, x):
        return self.layers(x)


class ResBlock2D(_Block):
    """x + NAC(NAC(x)) (modules.py:116-130); BN-apply+ReLU run in each conv's prologue and
    the residual add in the second conv's epilogue."""

    def __init__(self, in_channels, use_weight_norm):
        super().__init__()
        self.layers = nn.Sequential(
            ConvBlock2D("NAC", in_channels, in_channels, 3, 1, 1, use_weight_norm),
            ConvBlock2D("NAC", in_channels, in_channels, 3, 1, 1, use_weight_norm),
        )
        _ref(self, "bn1", self.layers[0].bn)
        _ref(self, "conv1", self.layers[0].conv)
        _ref(self, "bn2", self.layers[1].bn)
        _ref(self, "conv2", self.layers[1].conv)

    def forward(self, x):
        c1, c2 = self.conv1, self.conv2
        out = ops.ResBlockFn.apply(x, c1.weight_param(), c1.bias, self.bn1.weight, self.bn1.bias,
                                   c2.weight_param(), c2.bias, self.bn2.weight, self.bn2.bias, self)
        rec = getattr(self, "_fv_out_rec", None)
        if rec is not None:
            out._fv_bnrec = rec + (out._version,)     # the next ResBlock's bn1 statistics
            self._fv_out_rec = None
        q8 = getattr(self, "_fv_q8_consumer", None)
        if q8 is not None:
            out._fv_q8_consumer = q8                  # fp8: the conv consuming out's gradient
            self._fv_q8_consumer = None
        return out


class _Conv3(nn.Module):
    """Parameter holder of one nn.Conv3d(in, out, 3, 1, 1): `weight` [out][in][3][3][3] + `bias`,
    initialised as nn.Conv3d.reset_parameters (same RNG draws as the reference)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, bias=True):
        super().__init__()
        self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, kernel_size
        self.sn = False
        w = torch.empty(out_channels, in_channels, kernel_size, kernel_size, kernel_size)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        self.weight = nn.Parameter(w)
        if bias:
            bound = 1.0 / math.sqrt(in_channels * kernel_size ** 3)
            self.bias = nn.Parameter(torch.empty(out_channels).uniform_(-bound, bound))
        else:
            self.bias = None

    def weight_param(self):
        return self.weight

    def extra_repr(self):
        return f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}"


class ConvBlock3D(_Block):
    """_ConvBlock with dim=3 (modules.py:52-56): parameter / buffer holder with the reference
    state-dict keys.  It runs inside ResBlock3D ("NAC", 3x3x3, stride 1, padding 1); spectral
    norm and the other patterns raise."""

    def __init__(self, pattern, in_channels, out_channels, kernel_size, stride, padding, use_weight_norm,
                 activation_type="batch", nonlinearity_type="relu"):
        super().__init__()
        if (kernel_size, stride, padding) != (3, 1, 1) or pattern != "NAC" or use_weight_norm:
            raise NotImplementedError("facevae_amd ConvBlock3D: the ResBlock3D form only (NAC, 3x3x3, s1, p1, "
                                      "no spectral norm: AFE uses use_weight_norm=False, models.py:930)")
        if activation_type != "batch" or nonlinearity_type != "relu":
            raise NotImplementedError("facevae_amd ConvBlock3D: SyncBatchNorm + ReLU only")
        self.pattern = pattern
        mappings = {"C": _Conv3(in_channels, out_channels, kernel_size),
                    "N": _BatchNorm(in_channels),
                    "A": _Act(nonlinearity_type)}
        self.layers = nn.Sequential(*[mappings[c] for c in pattern])
        _ref(self, "conv", mappings["C"])
        _ref(self, "bn", mappings["N"])

    def forward(self, x):
        raise NotImplementedError("ConvBlock3D runs inside ResBlock3D (ops3d.ResBlock3DFn)")


class ResBlock3D(_Block):
    """x + NAC(NAC(x)) over [N, C, D, H, W] (modules.py:116-126, 133-135): 3x3x3 convs on
    the HIP kernels of conv3d.hip, BN/ReLU on the NHWC kernels over the NDHWC layout."""

    def __init__(self, in_channels, use_weight_norm):
        super().__init__()
        self.layers = nn.Sequential(
            ConvBlock3D("NAC", in_channels, in_channels, 3, 1, 1, use_weight_norm),
            ConvBlock3D("NAC", in_channels, in_channels, 3, 1, 1, use_weight_norm),
        )
        _ref(self, "bn1", self.layers[0].bn)
        _ref(self, "conv1", self.layers[0].conv)
        _ref(self, "bn2", self.layers[1].bn)
        _ref(self, "conv2", self.layers[1].conv)

    def forward(self, x):
        from . import ops3d
        c1, c2 = self.conv1, self.conv2
        return ops3d.ResBlock3DFn.apply(x, c1.weight, c1.bias, self.bn1.weight, self.bn1.bias,
                                        c2.weight, c2.bias, self.bn2.weight, self.bn2.bias, self)


class Conv2d(_Conv):
    """nn.Conv2d drop-in (stride 1, 'same' padding) with state-dict keys weight / bias."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        if stride != 1 or padding != kernel_size // 2:
            raise NotImplementedError("facevae_amd Conv2d: stride 1, 'same' padding only")
        super().__init__(in_channels, out_channels, kernel_size, False, bias)
        self._dtype = None

    def compute_dtype(self):
        return self._dtype or config.compute_dtype()

    def forward(self, x, sigmoid=False):
        return ops.ConvFn.apply(x, self.weight, self.bias, self, self.compute_dtype(), int(sigmoid))


class LinearELR(nn.Module):
    """LinearELR (models_utils.py:134-203) with act=None, norm=None: the style affine of a
    modulated ConvTranspose2dELR.  Same parameters and init draw; the tiny [B, wsize] x
    [wsize, outch] product runs as torch.addmm (alpha = weightgain), as the reference."""

    def __init__(self, inch, outch, lrmult=1., norm=None, act=None):
        super().__init__()
        if norm is not None or act is not None:
            raise NotImplementedError("LinearELR: norm=None, act=None only (the ConvTranspose2dELR affine)")
        self.weight = nn.Parameter(torch.randn(outch, inch) / lrmult)
        self.weightgain = 1. / math.sqrt(inch) * lrmult
        self.bias = nn.Parameter(torch.full([outch], 0.))

    def forward(self, x):
        return torch.addmm(self.bias[None], x, self.weight.t(), alpha=self.weightgain)


class ConvTranspose2dELR(nn.Module):
    """Drop-in for `ConvTranspose2dELR` (models_utils.py:404-516): a transposed conv with an
    equalised-learning-rate gain, optional per-output-channel weight demodulation and optional
    per-sample affine modulation (wsize > 0, forward(x, w)); same constructor, parameter names
    (`weight` [inch, outch, k, k], `bias`, `affine.weight/bias`) and init RNG draws
    (`blockinit(randn(inch, outch, k//s, k//s), s)`, models_utils.py:283-288, 435-446).

    Kernel size 4 / stride 2 / padding 1 at power-of-two sizes in bf16 runs on the sub-pixel
    MFMA kernels (ops.ConvTranspose2dFn); every other geometry, and fp32 parity mode, on the
    direct kernels of convt.hip (ops.ConvTranspose2dDirectFn).  Modulation is moved from the
    weights onto the activations: conv_t(x, W * s_b[i]) = conv_t(x * s_b, W), and the per-sample
    demodulation is an output-channel scale gain / ||W * s_b||_(i,r,s) (ops.ChanScaleFn); the
    [B, inch] / [B, outch] factors are formed with torch ops on those small tensors.  The untied
    bias (ub) and the activation module are applied after the kernel, as the reference does
    (models_utils.py:507-514)."""

    def __init__(self, inch, outch, kernel_size, stride, padding, wsize=0, affinelrmult=1., norm=None, ub=None,
                 act=None):
        super().__init__()
        self.inch, self.outch = inch, outch
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        self.wsize, self.norm, self.ub, self.act = wsize, norm, ub, act
        # models_utils.py:420-433: gain from the activation, then the init gain
        try:
            if isinstance(act, nn.LeakyReLU):
                actgain = nn.init.calculate_gain("leaky_relu", act.negative_slope)
            elif isinstance(act, nn.ReLU):
                actgain = nn.init.calculate_gain("relu")
            else:
                actgain = nn.init.calculate_gain(act)
        except Exception:
            actgain = 1.
        fan_in = inch * (kernel_size ** 2 / (stride ** 2))
        initgain = stride if norm == "demod" else 1. / math.sqrt(fan_in)
        self.weightgain = actgain * initgain
        k = kernel_size // stride
        w = torch.randn(inch, outch, k, k)
        self.weight = nn.Parameter(w.repeat_interleave(stride, dim=2).repeat_interleave(stride, dim=3).contiguous())
        self.bias = nn.Parameter(torch.zeros(outch, ub[0], ub[1]) if ub is not None else torch.zeros(outch))
        self.affine = LinearELR(wsize, inch, lrmult=affinelrmult) if wsize > 0 else None
        self.fused = False
        self._dtype = None

    def compute_dtype(self):
        return ops.storage(self._dtype or config.compute_dtype())

    def set_compute_dtype(self, dtype):
        self._dtype = dtype
        return self

    def extra_repr(self):
        return (f"inch={self.inch}, outch={self.outch}, kernel_size={self.kernel_size}, stride={self.stride}, "
                f"padding={self.padding}, wsize={self.wsize}, norm={self.norm}, ub={self.ub}, act={self.act}")

    def fuse(self):
        """Bake gain (and demodulation) into `weight` (models_utils.py:474-478)."""
        if self.affine is not None:
            return
        with torch.no_grad():
            w = self.weight
            if self.norm == "demod":
                w = F.normalize(w, dim=[0, 2, 3])
            self.weight.data = (w * self.weightgain).contiguous()
        self.fused = True

    def _core(self, x, bias, demod, gain, dtype):
        k, s, p = self.kernel_size, self.stride, self.padding
        if dtype == torch.bfloat16 and (k, s, p) == (4, 2, 1) and x.dim() == 4:
            N, inch, Hi, Wi = x.shape
            d = ops.desc(dtype, N, 2 * Hi, 2 * Wi, ops.pad_pow2(inch), inch, self.outch, self.outch, 3, ups=1)
            if ops.query("fv_convt_supported", ctypes.byref(d)):
                return ops.ConvTranspose2dFn.apply(x, self.weight, bias, demod, gain)
        return ops.ConvTranspose2dDirectFn.apply(x, self.weight, bias, k, s, p, demod, gain, dtype)

    def forward(self, x, w=None):
        dtype = self.compute_dtype()
        demod = self.norm == "demod" and not self.fused
        gain = 1.0 if self.fused else self.weightgain
        tied = self.bias.dim() == 1
        if self.affine is not None and w is not None:
            sb = self.affine(w) * 0.1 + 1.                          # [B, inch] (models_utils.py:488-489)
            if demod:                                               # per (b, o) over dims [1, 3, 4]
                wsq = (self.weight * self.weight).sum(dim=(2, 3))   # [inch, outch]
                scale = gain / torch.sqrt(torch.matmul(sb * sb, wsq)).clamp_min(1e-12)
            else:
                scale = torch.full((x.shape[0], self.outch), gain, device=x.device)
            xm = ops.ChanScaleFn.apply(x, sb, None, dtype)
            out = self._core(xm, None, False, 1.0, dtype)
            out = ops.ChanScaleFn.apply(out, scale, self.bias[None].expand(x.shape[0], -1) if tied else None, dtype)
        else:
            out = self._core(x, self.bias if tied else None, demod, gain, dtype)
        if not tied:
            out = out + self.bias[None].to(out.dtype)
        if self.act is not None:
            out = self.act(out)
        return out
