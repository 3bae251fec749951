"""PerceptualLoss (losses.py:123-151) on the HIP kernels: VGG19 and VGG-Face
feature stacks (torchvision `features` layouts, losses.py:53-120) whose 3x3 convs run on
conv.hip (fv_conv2d_fwd, and fv_conv2d_bwd_data for the input branch: the VGG weights are
frozen, losses.py:39-40, so no weight gradients are formed), ReLU / MaxPool2d / L1 on vgg.hip,
the per-channel normalisations (utils.py:182-193) and the 0.5x bilinear downscale of the
multi-scale loop (== 2x2 average on even sizes) on the BN/act kernels.

Same constructor arguments as the reference (layers_weight, n_scale) plus the feature-stack
weights: the reference downloads them by URL (vgg19-dcbb9e9d.pth, vgg_face_dag.pth,
losses.py:55-57, 80-82); there is no network here, so pass `vgg19_state_dict` /
`vggface_state_dict` ({"features.{i}.weight", "features.{i}.bias"}, torchvision numbering), or
ask explicitly for seeded random stacks with `random_init=True` (`width_div` narrows them for
tests); without either the constructor raises.  forward(input, target) follows
losses.py:131-151 exactly, including the multi-scale loop's reuse of the leaked `layer` /
`weight` (relu_5_1, 1.0) at every scale.  The target branch is computed without autograd (the
reference detaches it).  Activations are NHWC in the compute dtype (bf16 in fp8 mode).
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _lib as L
from . import config, ops
from ._lib import call, ptr, query, stream

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
VGG19_MAP = {1: "relu_1_1", 3: "relu_1_2", 6: "relu_2_1", 8: "relu_2_2", 11: "relu_3_1", 13: "relu_3_2",
             15: "relu_3_3", 17: "relu_3_4", 20: "relu_4_1", 22: "relu_4_2", 24: "relu_4_3", 26: "relu_4_4",
             29: "relu_5_1"}
VGG16_MAP = {1: "relu_1_1", 3: "relu_1_2", 6: "relu_2_1", 8: "relu_2_2", 11: "relu_3_1", 13: "relu_3_2",
             15: "relu_3_3", 18: "relu_4_1", 20: "relu_4_2", 22: "relu_4_3", 25: "relu_5_1"}
DEFAULT_WEIGHTS = {"relu_1_1": 0.03125, "relu_2_1": 0.0625, "relu_3_1": 0.125, "relu_4_1": 0.25, "relu_5_1": 1.0}
IMAGENET = ([0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
VGGFACE_MEAN = [129.186279296875, 104.76238250732422, 93.59396362304688]

F32 = torch.float32


def random_vgg_state(cfg, seed, width_div=1):
    """Seeded He-normal VGG feature weights (the stand-in when no downloaded stack is given)."""
    g = torch.Generator().manual_seed(seed)
    sd, cin, i = {}, 3, 0
    for v in cfg:
        if v == "M":
            i += 1
            continue
        co = v // width_div
        sd[f"features.{i}.weight"] = torch.randn(co, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
        sd[f"features.{i}.bias"] = torch.randn(co, generator=g) * 0.05
        cin, i = co, i + 2
    return sd


# ----------------------------------------------------------------------------------------
# autograd Functions on NHWC activations
# ----------------------------------------------------------------------------------------

class _ConvReLUFn(torch.autograd.Function):
    """relu(conv3x3(x) + b) with frozen weights: backward = ReLU mask then the data gradient."""

    @staticmethod
    def forward(ctx, x, w, b, dtype):
        N, cin, H, W = x.shape
        cout, cin_valid = w.shape[0], w.shape[1]
        d = ops.desc(dtype, N, H, W, cin, cin_valid, cout, cout, 3)
        wk = torch.empty(query("fv_conv_wk_elems", ctypes.byref(d)), dtype=dtype, device=x.device)
        wt = torch.empty(query("fv_conv_wt_elems", ctypes.byref(d)), dtype=dtype, device=x.device) \
            if ctx.needs_input_grad[0] else None
        call("fv_conv_weight_prep", ctypes.byref(d), ptr(w), None, ptr(wk), ptr(wt), stream())
        y = torch.empty((N, cout, H, W), dtype=dtype, device=x.device, memory_format=ops.CL)
        call("fv_conv2d_fwd", ctypes.byref(d), ptr(x), ptr(wk), ptr(b), None, None, None, ptr(y), None, stream())
        one = torch.ones(cout, dtype=F32, device=x.device)
        zero = torch.zeros(cout, dtype=F32, device=x.device)
        call("fv_bn_act_fwd", L.dtype_code(dtype), ptr(y), N, H, W, cout, cout, ptr(one), ptr(zero), 0.0, 0, ptr(y),
             stream())                                    # in-place ReLU
        ctx.d, ctx.wt, ctx.dtype = d, wt, dtype
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        d = ctx.d
        gb = ops.grad_in(g, ctx.dtype)
        gy = torch.empty_like(y)
        call("fv_relu_bwd", L.dtype_code(ctx.dtype), ptr(gb), ptr(y), y.numel(), ptr(gy), stream())
        dx = torch.empty((d.n, d.cin, d.h, d.w), dtype=ctx.dtype, device=y.device, memory_format=ops.CL)
        call("fv_conv2d_bwd_data", ctypes.byref(d), ptr(gy), d.cout, ptr(ctx.wt), ptr(dx), stream())
        return dx, None, None, None


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        N, C, H, W = x.shape
        y = torch.empty((N, C, H // 2, W // 2), dtype=dtype, device=x.device, memory_format=ops.CL)
        call("fv_maxpool2_fwd", L.dtype_code(dtype), ptr(x), N, H, W, C, ptr(y), stream())
        ctx.save_for_backward(x)
        ctx.dtype = dtype
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        N, C, H, W = x.shape
        if H % 2 or W % 2:
            raise RuntimeError("MaxPool2d backward: even input sizes only")
        dx = torch.empty_like(x)
        call("fv_maxpool2_bwd", L.dtype_code(ctx.dtype), ptr(x), ptr(ops.grad_in(g, ctx.dtype)), N, H, W, C, ptr(dx),
             stream())
        return dx, None


class _AffineFn(torch.autograd.Function):
    """per-channel x * scale + shift on an NHWC image (the normalisations), optionally followed
    by the 2x2 average (pool=1: F.interpolate 0.5x bilinear, align_corners=False, even sizes)."""

    @staticmethod
    def forward(ctx, x, scale, shift, pool, dtype):
        N, C, H, W = x.shape
        Ho, Wo = (H // 2, W // 2) if pool else (H, W)
        y = torch.empty((N, C, Ho, Wo), dtype=dtype, device=x.device, memory_format=ops.CL)
        call("fv_bn_act_fwd", L.dtype_code(dtype), ptr(x), N, H, W, C, C, ptr(scale), ptr(shift), 1.0, int(pool),
             ptr(y), stream())
        ctx.save_for_backward(scale)
        ctx.pool, ctx.dtype, ctx.shape = pool, dtype, (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, g):
        (scale,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        gb = ops.grad_in(g, ctx.dtype)
        if ctx.pool:
            up = torch.empty((N, C, H, W), dtype=ctx.dtype, device=g.device, memory_format=ops.CL)
            call("fv_avgpool2_bwd", L.dtype_code(ctx.dtype), ptr(gb), N, H, W, C, ptr(up), stream())
            gb = up
        dx = torch.empty_like(gb)
        zero = torch.zeros(C, dtype=F32, device=g.device)
        call("fv_bn_act_fwd", L.dtype_code(ctx.dtype), ptr(gb), N, H, W, C, C, ptr(scale), ptr(zero), 1.0, 0, ptr(dx),
             stream())
        return dx, None, None, None, None


class _L1Fn(torch.autograd.Function):
    """nn.L1Loss()(a, b.detach()) over NHWC feature tensors of one dtype."""

    @staticmethod
    def forward(ctx, a, b, dtype):
        out = torch.empty((), dtype=F32, device=a.device)
        ws = torch.empty(query("fv_l1t_ws_bytes") // 8, dtype=torch.float64, device=a.device)
        call("fv_l1t_fwd", L.dtype_code(dtype), ptr(a), ptr(b), a.numel(), ptr(out), ptr(ws), stream())
        ctx.save_for_backward(a, b)
        ctx.dtype = dtype
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        da = torch.empty_like(a)
        call("fv_l1t_bwd", L.dtype_code(ctx.dtype), ptr(a), ptr(b), a.numel(), ptr(g.float().contiguous()),
             1.0 / a.numel(), ptr(da), stream())
        return da, None, None


class _ImageFn(torch.autograd.Function):
    """NCHW fp32 image [N, 3, H, W] -> NHWC, 8 channels (zero padded), compute dtype."""

    @staticmethod
    def forward(ctx, x, dtype):
        xb, _ = ops.to_nhwc(x, dtype)
        ctx.shape, ctx.xdtype = x.shape, x.dtype
        return xb

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        out = torch.empty((N, C, H, W), dtype=F32, device=g.device)
        gb = g.contiguous(memory_format=ops.CL)
        call("fv_nhwc_to_nchw", L.dtype_code(gb.dtype), ptr(gb), N, C, H * W, gb.shape[1], ptr(out), stream())
        return out.to(ctx.xdtype), None


# ----------------------------------------------------------------------------------------
# modules
# ----------------------------------------------------------------------------------------

class VGGFeatures(nn.Module):
    """_PerceptualNetwork (losses.py:33-49) over a torchvision `features` stack: returns the
    activations named in `layers`, stopping after the last one needed."""

    def __init__(self, cfg, mapping, layers, state_dict):
        super().__init__()
        self.mapping, self.layers = dict(mapping), list(layers)
        self.kinds = []            # per torchvision index: ("conv", key) / ("relu",) / ("pool",)
        i = 0
        for v in cfg:
            if v == "M":
                self.kinds.append(("pool",))
                i += 1
            else:
                self.kinds += [("conv", i), ("relu",)]
                i += 2
        for k, v in state_dict.items():
            if k.startswith("features."):
                self.register_buffer(k.replace(".", "_"), v.detach().float().contiguous())
        self.last = max(i for i, n in self.mapping.items() if n in self.layers)

    def forward(self, x, dtype):
        out = {}
        i = 0
        while i <= self.last:
            kind = self.kinds[i]
            if kind[0] == "conv":
                w = getattr(self, f"features_{i}_weight")
                b = getattr(self, f"features_{i}_bias")
                x = _ConvReLUFn.apply(x, w, b, dtype)       # conv i and the ReLU at i + 1
                i += 1
            else:
                x = _MaxPoolFn.apply(x, dtype)
            if self.mapping.get(i) in self.layers:
                out[self.mapping[i]] = x
            i += 1
        return out


class PerceptualLoss(nn.Module):
    """Drop-in for losses.PerceptualLoss (losses.py:123-151); see the module docstring."""

    def __init__(self, layers_weight=None, n_scale=3, vgg19_state_dict=None, vggface_state_dict=None, width_div=1,
                 random_init=False):
        """vgg19_state_dict / vggface_state_dict: the pretrained feature stacks (torchvision
        layout) that the reference downloads by URL (losses.py:55-57, 80-82; unavailable
        offline).  Both are required unless `random_init=True` explicitly asks for seeded
        He-normal stand-ins (tests, benchmarks): a perceptual loss over random features is
        not the reference's loss, so it is never chosen silently."""
        super().__init__()
        self.layers_weight = dict(layers_weight or DEFAULT_WEIGHTS)
        self.n_scale = n_scale
        missing = [n for n, w in (("vgg19_state_dict", vgg19_state_dict), ("vggface_state_dict", vggface_state_dict))
                   if w is None]
        if missing and not random_init:
            raise ValueError(f"PerceptualLoss: {', '.join(missing)} not given -- pass the pretrained VGG weights "
                             "(torchvision layout) or random_init=True for seeded random feature stacks")
        w19 = vgg19_state_dict if vgg19_state_dict is not None else random_vgg_state(VGG19_CFG, 19, width_div)
        w16 = vggface_state_dict if vggface_state_dict is not None else random_vgg_state(VGG16_CFG, 16, width_div)
        self.vgg19 = VGGFeatures(VGG19_CFG, VGG19_MAP, self.layers_weight.keys(), w19)
        self.vggface = VGGFeatures(VGG16_CFG, VGG16_MAP, self.layers_weight.keys(), w16)
        self._dtype = None

    def compute_dtype(self):
        return ops.storage(self._dtype or config.compute_dtype())

    def set_compute_dtype(self, dtype):
        self._dtype = dtype
        return self

    def _affine(self, x, scale, shift, pool, dtype):
        C = x.shape[1]
        sc = torch.zeros(C, dtype=F32, device=x.device)
        sh = torch.zeros(C, dtype=F32, device=x.device)
        sc[:3] = torch.tensor(scale, dtype=F32)
        sh[:3] = torch.tensor(shift, dtype=F32)
        return _AffineFn.apply(x, sc, sh, pool, dtype)

    def forward(self, input, target):
        if not input.is_cuda:
            raise RuntimeError("facevae_amd ops run on the GPU only (HIP); got a CPU tensor")
        dt = self.compute_dtype()
        lw = self.layers_weight
        loss = ops.l1_loss(input, target.detach())                       # losses.py:137
        xi = _ImageFn.apply(input, dt)
        with torch.no_grad():
            xt = _ImageFn.apply(target.detach(), dt)
        face_s, face_b = [255.0] * 3, [-m for m in VGGFACE_MEAN]
        net_s = [1.0 / s for s in IMAGENET[1]]
        net_b = [-m / s for m, s in zip(*IMAGENET)]
        fi = self.vggface(self._affine(xi, face_s, face_b, 0, dt), dt)
        with torch.no_grad():
            ft = self.vggface(self._affine(xt, face_s, face_b, 0, dt), dt)
        ni = self._affine(xi, net_s, net_b, 0, dt)
        with torch.no_grad():
            nt = self._affine(xt, net_s, net_b, 0, dt)
            gt = self.vgg19(nt, dt)
        gi = self.vgg19(ni, dt)
        for layer, weight in lw.items():                                   # losses.py:142-144
            loss = loss + weight * _L1Fn.apply(fi[layer], ft[layer], dt) / 255
            loss = loss + weight * _L1Fn.apply(gi[layer], gt[layer], dt)
        one, zero = [1.0] * 3, [0.0] * 3
        for _ in range(self.n_scale):                                      # losses.py:145-150
            ni = self._affine(ni, one, zero, 1, dt)
            with torch.no_grad():
                nt = self._affine(nt, one, zero, 1, dt)
                gt = self.vgg19(nt, dt)
            gi = self.vgg19(ni, dt)
            loss = loss + weight * _L1Fn.apply(gi[layer], gt[layer], dt)   # leaked layer / weight
        return loss
