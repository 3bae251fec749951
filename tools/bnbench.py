"""BatchNorm streaming passes vs HBM: HIP-event time and achieved GB/s of each pass at the
step's shapes (bf16 NHWC), beside a plain device copy of the same tensor.

    python tools/bnbench.py [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import _lib as L, ops  # noqa: E402
from facevae_amd._lib import call, ptr, query, stream  # noqa: E402

CL = torch.channels_last


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    shapes = [(32, 256, 64, 64, 0), (32, 64, 256, 256, 0), (32, 128, 128, 128, 0), (32, 128, 256, 256, 1),
              (32, 256, 128, 128, 1)]
    for N, C, H, W, pool in shapes:
        bn = torch.nn.BatchNorm2d(C).cuda()
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.uniform_(-0.2, 0.2)
        y = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        Ho, Wo = (H // 2, W // 2) if pool else (H, W)
        dout = torch.randn(N, C, Ho, Wo, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        add = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        nbytes = y.numel() * 2
        r = ops.bn_from_tensor(bn, y, True, None)
        t = {}
        t["copy"] = (timeit(lambda: y.clone(), a.iters), 2 * nbytes)
        t["stats"] = (timeit(lambda: ops.bn_from_tensor(bn, y, True, None), a.iters), nbytes)
        t["act_fwd"] = (timeit(lambda: ops.bn_act_forward(y, r, 0.0, pool, bn), a.iters),
                        nbytes + nbytes // (4 if pool else 1))
        dev = y.device
        ws = torch.empty(query("fv_bn_ws_bytes", C) // 8, dtype=torch.float64, device=dev)
        dg = torch.empty(C, device=dev)
        dbt = torch.empty(C, device=dev)
        k = torch.empty(2 * C, device=dev)
        dc = L.dtype_code(y.dtype)
        dx = torch.empty_like(y)

        def red():
            call("fv_bn_act_bwd_reduce_finalize", dc, ptr(dout), ptr(y), N, H, W, C, C, ptr(r.mean), ptr(r.invstd),
                 ptr(bn.weight), ptr(bn.bias), 0.0, int(pool), int(r.count), ptr(dg), ptr(dbt), ptr(k), ptr(ws), stream())

        def app(addend):
            call("fv_bn_act_bwd_apply", dc, ptr(dout), ptr(y), N, H, W, C, C, ptr(r.mean), ptr(r.invstd),
                 ptr(bn.weight), ptr(bn.bias), 0.0, int(pool), ptr(k), ptr(addend), ptr(dx), stream())
        t["bwd_reduce"] = (timeit(red, a.iters), nbytes + dout.numel() * 2)
        t["bwd_apply"] = (timeit(lambda: app(None), a.iters), 2 * nbytes + dout.numel() * 2)
        if not pool:
            t["bwd_apply+add"] = (timeit(lambda: app(add), a.iters), 3 * nbytes + dout.numel() * 2)
        print(f"N{N} C{C} {H}x{W}{' pool' if pool else ''}: " +
              "  ".join(f"{k_} {us:.1f}us {b / us / 1e3:.2f}GB/s" for k_, (us, b) in t.items()), flush=True)


if __name__ == "__main__":
    main()
