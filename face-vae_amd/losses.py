"""Loss modules with the reference call signatures (losses.py of Luh1124/face-vae)."""
from __future__ import annotations

from torch import nn

from . import ops


class KLDivergenceLoss(nn.Module):
    """losses.py:385-393: mean(-0.5 - logstd + 0.5 mu^2 + 0.5 exp(2 logstd)); called as
    KLDivergenceLoss()((mu, logstd))."""

    def forward(self, kl):
        return ops.kl_loss(kl[0], kl[1])


class ReconLoss(nn.Module):
    """losses.py:396-403: nn.MSELoss()(Rec[0], Rec[1]); called as ReconLoss()((target, pred))."""

    def forward(self, Rec):
        return ops.mse_loss(Rec[0], Rec[1])


class L1Loss(nn.Module):
    """nn.L1Loss (mean |a - b|): the pixel term of PerceptualLoss (losses.py:128,135)."""

    def forward(self, input, target):
        return ops.l1_loss(input, target)


from .perceptual import PerceptualLoss  # noqa: E402,F401  (losses.py:123-151)
