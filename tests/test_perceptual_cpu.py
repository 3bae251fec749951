"""Perceptual loss on the CPU: the oracle restatement against the reference's
own PerceptualLoss.forward run over seeded narrow VGG stacks (tests/golden/make_golden_perceptual.py)."""
import os
import sys

import torch

from oracle import facevae_cpu as O

HERE = os.path.dirname(__file__)
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_golden_perceptual import (VGG16_CFG, VGG19_CFG, perceptual_images,  # noqa: E402
                                    perceptual_weights)


def test_perceptual_oracle_matches_reference():
    g = torch.load(os.path.join(HERE, "golden", "perceptual.pt"), weights_only=True)
    w19, w16 = perceptual_weights(VGG19_CFG, 101), perceptual_weights(VGG16_CFG, 102)
    assert abs(sum(v.double().sum() for v in w19.values()).item() - g["w19_sum"].item()) < 1e-9
    assert abs(sum(v.double().sum() for v in w16.values()).item() - g["w16_sum"].item()) < 1e-9
    x, t = perceptual_images()
    assert abs(x.double().sum().item() - g["x_sum"].item()) < 1e-9
    xr = x.clone().requires_grad_(True)
    loss = O.perceptual_loss(xr, t, w19, w16)
    loss.backward()
    assert abs(loss.item() - g["loss"].item()) / g["loss"].item() < 1e-6
    d = ((xr.grad.double() - g["d_input"].double()).norm() / g["d_input"].double().norm()).item()
    assert d < 1e-5


def test_perceptual_loss_needs_weights_or_explicit_random_init():
    """the drop-in PerceptualLoss never silently trains against random features."""
    import pytest
    import fvamd  # noqa: F401
    import facevae_amd as fv
    with pytest.raises(ValueError, match="random_init=True"):
        fv.PerceptualLoss()
    with pytest.raises(ValueError, match="vggface_state_dict"):
        fv.PerceptualLoss(vgg19_state_dict=perceptual_weights(VGG19_CFG, 101))
    crit = fv.PerceptualLoss(random_init=True, width_div=16)
    assert crit.vgg19.last > 0 and crit.vggface.last > 0
