"""Encoder (AFE 2-D trunk), decoder (Generator 2-D trunk) and the FaceVAE composition
 with the reference constructor signatures and state-dict keys
(models.py:922-945 AFE, 1085-1111 Generator of Luh1124/face-vae)."""
from __future__ import annotations

import torch
from torch import nn

from . import config as _config
from . import ops
from . import ops3d, warp
from .modules import Conv2d, ConvBlock2D, DownBlock2D, ResBlock2D, ResBlock3D, UpBlock2D, _Block


def _batched_weight_prep(model, device):
    """The per-step weight work of every conv under `model` in a few launches: one batched
    power iteration for the spectral-normed convs (ops.SNBatch, 4 launches for all of them) and
    one re-layout launch for the generic weight layouts (ops.WPrepBatch).  Run by the top-level
    forward of AFE / Generator / FaceVAE (sub-module calls go through forward_2d)."""
    from .modules import _Conv
    sb = model.__dict__.get("_snb")
    if sb is None:
        sb = ops.SNBatch([c for c in model.modules() if isinstance(c, _Conv) and c.sn])
        object.__setattr__(model, "_snb", sb)
    wb = model.__dict__.get("_wpb")
    if wb is None:
        wb = ops.WPrepBatch([c for c in model.modules() if isinstance(c, _Conv)])
        object.__setattr__(model, "_wpb", wb)
    sb.run(model.training)
    wb.run(device)


class AFE(_Block):
    """Appearance-feature extractor (models.py:922-945): in_conv 7x7 CNA, DownBlock2D chain,
    1x1 mid_conv (the 2-D trunk = the FaceVAE encoder), then x.view(N, C, D, H, W) and n_res
    ResBlock3D(C) (the 3-D trunk).  forward(x) -> [N, C, D, H/4, W/4] in the compute dtype,
    NDHWC memory (torch.channels_last_3d)."""

    def __init__(self, use_weight_norm=False, down_seq=(64, 128, 256), n_res=6, C=32, D=16):
        super().__init__()
        down_seq = list(down_seq)
        self.in_conv = ConvBlock2D("CNA", 3, down_seq[0], 7, 1, 3, use_weight_norm)
        self.down = nn.Sequential(*[DownBlock2D(down_seq[i], down_seq[i + 1], use_weight_norm)
                                    for i in range(len(down_seq) - 1)])
        self.mid_conv = Conv2d(down_seq[-1], C * D, 1, 1, 0)
        self.res = nn.Sequential(*[ResBlock3D(C, use_weight_norm) for _ in range(n_res)])
        self.C, self.D = C, D

    def forward_2d(self, x):
        return self.mid_conv(self.down(self.in_conv(x)))

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("facevae_amd ops run on the GPU only (HIP); got a CPU tensor")
        _batched_weight_prep(self, x.device)
        h = self.forward_2d(x)
        fs = ops3d.depth_split(h, self.C, self.D, self.compute_dtype())
        if len(self.res):
            wb = self.__dict__.get("_w3b")
            if wb is None:
                wb = ops3d.W3PrepBatch([c for blk in self.res for c in (blk.conv1, blk.conv2)])
                object.__setattr__(self, "_w3b", wb)
            N, C, D, H, W = fs.shape
            wb.prep(ops3d.desc3(ops.storage(self.compute_dtype()), N, D, H, W, C, C), x.device)
        return self.res(fs)


class Generator(_Block):
    """Decoder (models.py:1085-1111): grid_sample of the 3-D appearance volume by the motion
    field (1103, warp.grid_sample_3d), view to [N, C*D, H, W], in_conv (SN, LeakyReLU .2),
    mid_conv, occlusion multiply (1106, warp.occlusion_multiply), 6 ResBlock2D, 2 UpBlock2D,
    out_conv 7x7 + sigmoid.  forward(fs, deformation=None, occlusion=None): None skips the warp
    / the occlusion (identity), which is the FaceVAE composition's 2-D input."""

    def __init__(self, use_weight_norm=True, n_res=6, up_seq=(256, 128, 64), D=16, C=32):
        super().__init__()
        up_seq = list(up_seq)
        self.in_conv = ConvBlock2D("CNA", C * D, up_seq[0], 3, 1, 1, use_weight_norm, nonlinearity_type="leakyrelu")
        self.mid_conv = Conv2d(up_seq[0], up_seq[0], 1, 1, 0)
        self.res = nn.Sequential(*[ResBlock2D(up_seq[0], use_weight_norm) for _ in range(n_res)])
        self.up = nn.Sequential(*[UpBlock2D(up_seq[i], up_seq[i + 1], use_weight_norm)
                                  for i in range(len(up_seq) - 1)])
        self.out_conv = Conv2d(up_seq[-1], 3, 7, 1, 3)

    def forward_2d(self, fs, occlusion=None):
        fs = self.in_conv(fs)
        fs = self.mid_conv(fs)
        if occlusion is not None:
            fs = warp.occlusion_multiply(fs, occlusion, self.compute_dtype())
        fs = self.res(fs)
        fs = self.up(fs)
        return self.out_conv(fs, sigmoid=True)       # conv + bias + sigmoid, NCHW fp32 out

    def forward(self, fs, deformation=None, occlusion=None):
        mode = self.compute_dtype()
        if fs.is_cuda:
            _batched_weight_prep(self, fs.device)
        if fs.dim() == 5:
            if deformation is not None:
                fs = warp.grid_sample_3d(fs, deformation, ops.storage(mode))
            fs = ops3d.depth_merge(fs, mode)          # .view(N, -1, H, W), models.py:1103
        elif deformation is not None:
            raise ValueError("Generator: a deformation needs the 5-D feature volume fs [N, C, D, H, W]")
        return self.forward_2d(fs, occlusion)


class FaceVAE(_Block):
    """AFE 2-D trunk -> [mu | logstd] split + reparameterisation -> Generator 2-D trunk.

    forward(x, eps) -> (y, mu, logstd).  x: [B,3,H,H] fp32 in [0,1]; eps: [B,L,H/4,H/4]
    standard-normal noise (the reference draws it with torch.randn inside
    flatten_vae_nl, models.py:561; here it is an input so runs are reproducible)."""

    def __init__(self, cfg: _config.FaceVAEConfig = None):
        super().__init__()
        cfg = cfg or _config.FaceVAEConfig()
        self.cfg = cfg
        self.afe = AFE(False, list(cfg.down_seq), 0, C=2 * cfg.latent, D=1)
        self.generator = Generator(True, cfg.n_res, list(cfg.up_seq), D=1, C=cfg.latent)

    def forward(self, x, eps):
        if x.is_cuda:
            # all 15 power iterations in 4 launches, the generic weight layouts in one
            _batched_weight_prep(self, x.device)
        h = self.afe.forward_2d(x)
        mu, logstd, z = ops.reparameterise(h, eps, self.compute_dtype())
        y = self.generator.forward_2d(z)
        return y, mu, logstd
