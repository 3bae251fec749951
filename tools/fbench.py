"""SURVEY §8(f) path benchmark: the reference's full-size decoder input path as one training
step -- AFE() (models.py:928-945: 2-D trunk + x.view(N, 32, 16, 64, 64) + 6 ResBlock3D) ->
Generator()(fs, deformation, occlusion) (models.py:1101-1111: grid_sample warp, in_conv,
mid_conv, occlusion multiply, 6 ResBlock2D, 2 UpBlock2D, out_conv + sigmoid) -> MSE to a
target image -> backward -> Adam, on synthetic inputs resident in HBM (x ~ U[0,1), an identity
sampling grid + 0.05 N(0,1), sigmoid(N(0,1)) occlusion; seed-0 random init).  This is the path
trainer.py:268, 296-297 runs without the keypoint / pose nets.

    python tools/fbench.py [--batch 8] [--steps 10] [--warmup 3] [--dtype bf16] [--graph 1]

Prints ONE JSON line: images/s, ms/step, the algorithmic FLOPs of the step (reference
formulation), the step's bf16-MFMA utilisation, and the HIP-event durations of the 3-D
convolutions (fwd / dgrad / wgrad) measured over eager steps after the timed region.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import ops3d, warp  # noqa: E402

PEAK_BF16_TFLOPS = 2516.6


def conv_flops(h, w, cin, cout, k, d=1, kd=1):
    return 2.0 * d * h * w * cin * cout * k * k * kd


def step_flops_per_image(H=256, down=(64, 128, 256), C=32, D=16, n_res3=6, up=(256, 128, 64), n_res2=6):
    """Reference-formulation FLOPs of one training step per image (fwd x 3, minus the input
    conv's data gradient), the 3-D part separately."""
    q = H // 4
    f2 = conv_flops(H, H, 3, down[0], 7)                                   # AFE.in_conv
    res = H
    for i in range(len(down) - 1):                                         # DownBlock2D: conv at input res
        f2 += conv_flops(res, res, down[i], down[i + 1], 3)
        res //= 2
    f2 += conv_flops(q, q, down[-1], C * D, 1)                             # AFE.mid_conv
    f3 = n_res3 * 2 * conv_flops(q, q, C, C, 3, d=D, kd=3)                 # ResBlock3D x 6
    f2 += conv_flops(q, q, C * D, up[0], 3)                                # Generator.in_conv
    f2 += conv_flops(q, q, up[0], up[0], 1)                                # Generator.mid_conv
    f2 += n_res2 * 2 * conv_flops(q, q, up[0], up[0], 3)                   # ResBlock2D x 6
    res = q
    for i in range(len(up) - 1):                                           # UpBlock2D: conv at output res
        res *= 2
        f2 += conv_flops(res, res, up[i], up[i + 1], 3)
    f2 += conv_flops(H, H, up[-1], 3, 7)                                   # out_conv
    in_dgrad = conv_flops(H, H, 3, down[0], 7)
    return 3 * (f2 + f3) - in_dgrad, 3 * f3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--graph", type=int, default=1)
    a = ap.parse_args()
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype]
    B, H = a.batch, 256
    torch.manual_seed(0)
    afe = fv.AFE().cuda().train().set_compute_dtype(dtype)
    gen = fv.Generator().cuda().train().set_compute_dtype(dtype)
    params = list(afe.parameters()) + list(gen.parameters())
    opt = fv.Adam(params, lr=5e-5, betas=(0.5, 0.999))
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(B, 3, H, H, generator=g).cuda()
    target = torch.rand(B, 3, H, H, generator=g).cuda()
    ident = warp.make_coordinate_grid_3d((16, H // 4, H // 4))[None]
    deform = (ident + 0.05 * torch.randn(B, 16, H // 4, H // 4, 3, generator=g)).cuda()
    occ = torch.sigmoid(torch.randn(B, 1, H // 4, H // 4, generator=g)).cuda()
    rec = fv.ReconLoss()

    def step():
        opt.zero_grad(set_to_none=True)
        fs = afe(x)
        y = gen(fs, deform, occ)
        loss = rec((target, y))
        loss.backward()
        opt.step()
        return loss

    # 3-D conv launch durations (HIP events on the launch stream, eager steps only)
    events = {}
    orig = {k: getattr(ops3d, k) for k in ("conv3d_forward", "conv3d_backward") if hasattr(ops3d, k)}

    def timed(name, fn):
        def w(*args, **kw):
            if torch.cuda.is_current_stream_capturing() or not timing[0]:
                return fn(*args, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*args, **kw)
            e1.record()
            events.setdefault(name, []).append((e0, e1))
            return r
        return w
    timing = [False]
    for k, fn in orig.items():
        setattr(ops3d, k, timed(k, fn))

    step()
    run = step
    if a.graph:
        sg = fv.StepGraph(step, [opt], warmup=max(1, a.warmup - 1)).capture()
        run = sg.replay
        for _ in range(2):
            run()
    else:
        for _ in range(a.warmup - 1):
            step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = run()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    timing[0] = True
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    timing[0] = False
    assert torch.isfinite(loss).item()
    ev = {k: sum(e0.elapsed_time(e1) for e0, e1 in v) / len(v) for k, v in events.items() if v}
    f_img, f3 = step_flops_per_image(H)
    ips = B * a.steps / t
    out = {
        "metric": "training images/sec (256x256 AFE() 3-D trunk -> warp -> Generator() step, SURVEY 8(f))",
        "value": round(ips, 2), "unit": "images/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(t / a.steps * 1e3, 3), "higher_is_better": True, "dtype": a.dtype,
        "data": "synthetic (x, target ~ U[0,1), deformation = identity + 0.05 N(0,1), occlusion = sigmoid(N(0,1)); "
                "seed-0 random init)",
        "config": {"workload": "AFE() -> grid_sample -> Generator(), MSE, Adam", "batch": B, "resolution": H,
                   "launch": "hip graph" if a.graph else "eager"},
        "step_flop_per_image": f_img, "conv3d_flop_per_image": f3,
        "mfma_util_step": round(ips * f_img / (PEAK_BF16_TFLOPS * 1e12), 4),
        "conv3d_wrapper_avg_ms": {k: round(v, 4) for k, v in ev.items()},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
