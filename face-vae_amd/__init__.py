"""facevae_amd — MI355X-native (gfx950) FaceVAE training step.

Import as `facevae_amd` (see `load_package()` in the repo root's __graft_entry__.py, or
`import fvamd` which registers the package under that name).

Hot path: AFE 2-D trunk -> latent split/reparam -> Generator 2-D trunk,
MSE + KL, Adam; every compute op is a hand-written HIP kernel in libfacevae.so called
through the C-ABI in include/facevae.h.
"""
from . import _lib
from .config import FaceVAEConfig, compute_dtype, set_compute_dtype
from .losses import KLDivergenceLoss, L1Loss, PerceptualLoss, ReconLoss
from .models import AFE, FaceVAE, Generator
from .modules import (Conv2d, ConvBlock2D, ConvBlock3D, ConvTranspose2dELR, DownBlock2D, ResBlock2D, ResBlock3D,
                      SameBlock2D, UpBlock2D)
from .optim import Adam
from . import checkpoint, distributed, graph, ops, ops3d, warp
from .graph import StepGraph

__all__ = ["FaceVAEConfig", "compute_dtype", "set_compute_dtype", "KLDivergenceLoss", "L1Loss", "PerceptualLoss", "ReconLoss",
           "AFE", "FaceVAE", "Generator", "Conv2d", "ConvBlock2D", "ConvTranspose2dELR", "DownBlock2D", "ResBlock2D", "ResBlock3D", "ConvBlock3D", "SameBlock2D",
           "UpBlock2D", "Adam", "distributed", "ops", "FaceVAETrainer"]


def __getattr__(name):
    if name == "FaceVAETrainer":
        from .trainer import FaceVAETrainer
        return FaceVAETrainer
    raise AttributeError(name)
