"""Diagnostic: per-parameter gradient deviation of the full-size Generator() 2-D trunk in
fp32 parity mode vs the CPU oracle (B=1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from oracle import facevae_cpu as O  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    H = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    torch.manual_seed(3)
    gen = fv.Generator()
    sd = O.prepare_state({f"generator.{k}": v for k, v in gen.state_dict().items()})
    g = torch.Generator().manual_seed(4)
    z = torch.randn(1, 512, H, H, generator=g)
    gen = gen.cuda().train().set_compute_dtype(torch.float32)
    y = gen(z.cuda())
    gy = torch.randn(y.shape, generator=g)
    (y * gy.cuda()).sum().backward()
    torch.cuda.synchronize()
    cfg = O.OracleConfig(H=4 * H)
    yo = O.decode(sd, z, cfg, True)
    (yo * gy).sum().backward()
    print("image", rel(y, yo))
    for k, p in gen.named_parameters():
        if not k.endswith("bias"):
            print(f"{rel(p.grad, sd['generator.' + k].grad):.2e} {k}")


if __name__ == "__main__":
    main()
