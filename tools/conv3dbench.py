"""Per-kernel timing of the AFE 3-D trunk convs (conv3d.hip) at the reference shape
[B, 32, 16, 64, 64] (AFE C=32, D=16 at 256x256 input), bf16, plus one ResBlock3D fwd+bwd.

    python tools/conv3dbench.py [--batch 32] [--iters 20]

FLOPs per conv launch = 2 * B*16*64*64 voxels * 32 * 32 * 27 (fwd, dgrad and wgrad alike).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import ops3d  # noqa: E402

PEAK = 2516.6


class _W:
    def __init__(self, w):
        self.weight = w


def timeit(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    B = a.batch
    shape = (B, 32, 16, 64, 64)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(shape, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=ops3d.CL3)
    dy = torch.randn(shape, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=ops3d.CL3)
    w = (torch.randn(32, 32, 3, 3, 3, generator=g) * 0.05).cuda()
    b = torch.zeros(32, device="cuda")
    d = ops3d.desc3(torch.bfloat16, B, 16, 64, 64, 32, 32)
    cs = ops3d.Conv3dState(_W(w), d, "cuda", True)
    flop = 2.0 * B * 16 * 64 * 64 * 32 * 32 * 27
    out = {"shape": list(shape), "flop_per_launch": flop}
    t = timeit(lambda: ops3d.conv3d_forward(cs, x, b, stats=True), a.iters)
    out["fwd_ms"] = round(t, 4)
    t = timeit(lambda: ops3d.conv3d_backward(cs, x, dy, need_dx=True), a.iters)
    out["dgrad_plus_wgrad_ms"] = round(t, 4)
    t2 = timeit(lambda: ops3d.conv3d_backward(cs, x, dy, need_dx=False), a.iters)
    out["wgrad_ms"] = round(t2, 4)
    out["dgrad_ms"] = round(t - t2, 4)
    for k in ("fwd", "wgrad", "dgrad"):
        out[k + "_tflops"] = round(flop / (out[k + "_ms"] * 1e-3) / 1e12, 1)
        out[k + "_frac_bf16_peak"] = round(out[k + "_tflops"] / PEAK, 4)
    blk = fv.ResBlock3D(32, False).cuda().train().set_compute_dtype(torch.bfloat16)
    xr = x.detach().clone().requires_grad_(True)

    def step():
        y = blk(xr)
        y.backward(dy)
    out["resblock3d_fwd_bwd_ms"] = round(timeit(step, a.iters), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
