"""Checkpoint interchange with reference `Logger` runs (logger.py:92-115 of Luh1124/face-vae).

`Logger.save_cpk` writes ONE dict per epoch to `<ckp_dir>/%08d-checkpoint.pth.tar`:
`{name: model.module.state_dict()}` for the generator-side models `efe, afe, ckd, hpe_ede, mfe,
generator` and `discriminator` (no "module." prefix: the DDP wrapper is unwrapped), plus
`"optimizer_" + name` (torch.optim.Adam state dicts, betas (0.5, 0.999)) and `"epoch"`.  The
models are the full-size `AFE()` (models.py:922-945: 2-D trunk + 6 ResBlock3D, C=32, D=16) and
`Generator()` (models.py:1085-1111: in_conv 512 -> 256 with spectral norm, ...), SyncBatchNorm
converted (same state-dict keys as BatchNorm).

This module reads and writes that layout for the two models this repo implements:

* `load_reference_checkpoint(path)` -> `{"afe": AFE(), "generator": Generator(), "epoch": e,
  "optimizer_afe": ..., "optimizer_generator": ...}`: our full-size modules (same constructor
  defaults, same key set and shapes -- pinned against the reference in
  tests/golden/module_keys.json) with the reference weights / buffers loaded strictly, and the
  reference Adam states as state dicts our `Adam` (torch.optim.Adam layout) loads as they are.
* `save_reference_checkpoint(path, afe, generator, optimizers, epoch)` writes the same layout
  (only these two models; a reference Logger.load_cpk needs the other five as well).

Loading uses `torch.load(weights_only=True)`: a checkpoint is data, nothing in it executes.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch

from .models import AFE, Generator

MODELS = ("afe", "generator")


def reference_checkpoint_path(ckp_dir: str, epoch: int, zfill_num: int = 8) -> str:
    """logger.py:101,105: the file Logger.save_cpk writes for `epoch`."""
    return os.path.join(ckp_dir, "%s-checkpoint.pth.tar" % str(epoch).zfill(zfill_num))


def _strict_load(module: torch.nn.Module, sd: Dict[str, torch.Tensor], name: str):
    own = module.state_dict()
    missing = sorted(set(own) - set(sd))
    extra = sorted(set(sd) - set(own))
    if missing or extra:
        raise KeyError(f"reference checkpoint[{name!r}]: keys differ from {type(module).__name__}() "
                       f"(missing {missing[:4]}{'...' if len(missing) > 4 else ''}, "
                       f"unexpected {extra[:4]}{'...' if len(extra) > 4 else ''})")
    for k, v in sd.items():
        if tuple(own[k].shape) != tuple(v.shape):
            raise ValueError(f"reference checkpoint[{name!r}][{k!r}]: shape {tuple(v.shape)}, "
                             f"{type(module).__name__}() has {tuple(own[k].shape)}")
    module.load_state_dict(sd, strict=True)


def load_reference_checkpoint(path: str, afe: Optional[AFE] = None, generator: Optional[Generator] = None,
                              map_location="cpu") -> Dict[str, object]:
    """Load the `afe` / `generator` entries of a reference Logger checkpoint into full-size
    AFE() / Generator() modules (new ones unless given).  Raises if a key or shape differs."""
    ckp = torch.load(path, map_location=map_location, weights_only=True)
    for name in MODELS:
        if name not in ckp:
            raise KeyError(f"{path}: no {name!r} entry (keys: {sorted(ckp)[:8]})")
    afe = afe if afe is not None else AFE()
    generator = generator if generator is not None else Generator()
    _strict_load(afe, ckp["afe"], "afe")
    _strict_load(generator, ckp["generator"], "generator")
    out = {"afe": afe, "generator": generator, "epoch": ckp.get("epoch")}
    for name in MODELS:
        if "optimizer_" + name in ckp:
            out["optimizer_" + name] = ckp["optimizer_" + name]
    return out


def save_reference_checkpoint(path: str, afe: AFE, generator: Generator, optimizers: Optional[Dict] = None,
                              epoch: int = 0):
    """Write afe / generator (+ their Adam states) in Logger.save_cpk's layout."""
    ckp = {"afe": afe.state_dict(), "generator": generator.state_dict()}
    for name, opt in (optimizers or {}).items():
        ckp["optimizer_" + name] = opt.state_dict()
    ckp["epoch"] = epoch
    torch.save(ckp, path)
