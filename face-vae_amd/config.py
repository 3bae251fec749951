"""Run-time configuration: compute dtype and the FaceVAE composition shapes."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch

_COMPUTE_DTYPE = torch.bfloat16


def compute_dtype() -> torch.dtype:
    return _COMPUTE_DTYPE


COMPUTE_MODES = (torch.float32, torch.bfloat16, torch.float8_e4m3fn)


def set_compute_dtype(dtype: torch.dtype) -> None:
    """torch.float32 = exact-fp32 MFMA parity mode; torch.bfloat16 = bf16 MFMA (default);
    torch.float8_e4m3fn = bf16 activations with the 3x3 convs' forward and data gradient on
    per-tensor scaled e4m3 operands (BASELINE config C5)."""
    global _COMPUTE_DTYPE
    if dtype not in COMPUTE_MODES:
        raise ValueError("compute dtype must be torch.float32, torch.bfloat16 or torch.float8_e4m3fn")
    _COMPUTE_DTYPE = dtype


@dataclass
class FaceVAEConfig:
    """Shapes of the FaceVAE composition: AFE 2-D trunk -> latent split /
    reparam -> Generator 2-D trunk.  Defaults = the 256x256 reference shapes."""
    H: int = 256
    down_seq: Tuple[int, ...] = (64, 128, 256)
    latent: int = 256
    n_res: int = 6
    up_seq: Tuple[int, ...] = (256, 128, 64)
    w_R: float = 1.0          # ReconLoss weight (reference comment: 10, trainer.py:251)
    w_K: float = 1.0          # KL weight (reference comment: 0.2, trainer.py:250)
    lr: float = 5e-5          # train.py:34
    betas: Tuple[float, float] = (0.5, 0.999)   # logger.py:60
    syncbn: bool = True       # SyncBatchNorm semantics across ranks (logger.py:55)

    @staticmethod
    def toy() -> "FaceVAEConfig":
        return FaceVAEConfig(H=64, down_seq=(16, 32), latent=16, n_res=1, up_seq=(32, 16))

    @staticmethod
    def hires() -> "FaceVAEConfig":
        return FaceVAEConfig(H=512)

    @property
    def latent_hw(self) -> int:
        return self.H >> (len(self.down_seq) - 1)
