"""Generate the golden fixtures of the AFE 3-D trunk FROM THE REFERENCE ITSELF.

Run in the build container only (it needs /root/reference, absent on the GPU box):

    python tests/golden/make_golden_3d.py

Imports the reference `modules.py` / `models.py` read-only (see make_golden.py) and stores
plain tensors in tests/golden/afe3d.pt (loaded with weights_only=True):

  res3d   ResBlock3D(32, use_weight_norm=False) (modules.py:133-135) in training mode on
          x [1, 32, 4, 4, 64]: output, input gradient and parameter gradients for the
          upstream gradient g, BN running statistics after the step, and the eval-mode
          output with those statistics.
  afe3d   AFE(use_weight_norm=False, down_seq=[16, 32], n_res=1, C=32, D=2) (models.py:922-945)
          in training mode on x [2, 3, 64, 64]: the [2, 32, 2, 32, 32] output and every
          parameter gradient of sum(out * g).
Initial parameters are not stored: the product modules draw the same RNG sequence as the
reference constructors, so torch.manual_seed(seed) + construction reproduces them (the test
checks a checksum of each).
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference  # noqa: E402


def grads(mod):
    return {k: p.grad.detach().clone() for k, p in mod.named_parameters()}


def main():
    modules, models, _ = import_reference()
    torch.set_num_threads(8)
    out = {}

    torch.manual_seed(11)
    blk = modules.ResBlock3D(32, False).train()
    init_sum = {k: v.detach().double().sum() for k, v in blk.state_dict().items() if v.is_floating_point()}
    x = torch.randn(1, 32, 4, 4, 64, generator=torch.Generator().manual_seed(12))
    g = torch.randn(1, 32, 4, 4, 64, generator=torch.Generator().manual_seed(13))
    xr = x.clone().requires_grad_(True)
    y = blk(xr)
    (y * g).sum().backward()
    bufs = {k: v.detach().clone() for k, v in blk.state_dict().items() if "running" in k or "num_batches" in k}
    blk.eval()
    with torch.no_grad():
        y_eval = blk(x)
    out["res3d"] = dict(seed=torch.tensor(11), x=x, g=g, out=y.detach(), dx=xr.grad.detach(), grads=grads(blk),
                        buffers=bufs, out_eval=y_eval, init_sum=init_sum)

    torch.manual_seed(21)
    afe = models.AFE(use_weight_norm=False, down_seq=[16, 32], n_res=1, C=32, D=2).train()
    init_sum = {k: v.detach().double().sum() for k, v in afe.state_dict().items() if v.is_floating_point()}
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(22))
    y = afe(x)
    g = torch.randn(y.shape, generator=torch.Generator().manual_seed(23))
    (y * g).sum().backward()
    out["afe3d"] = dict(seed=torch.tensor(21), x=x, g=g, out=y.detach(), grads=grads(afe), init_sum=init_sum)

    path = os.path.join(HERE, "afe3d.pt")
    torch.save(out, path)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
