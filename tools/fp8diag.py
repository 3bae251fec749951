"""Diagnostic: the fp8 weight gradient of every eligible conv in a B-image fp8 step, re-run in
isolation on the same e4m3 operands and on fresh copies of them, against float64."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import _lib as L, ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def run_wg(d, x8, xdq, dy8, dydq):
    slab = torch.zeros(L.query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), device="cuda")
    bslab = torch.zeros(L.query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), device="cuda")
    L.call("fv_conv2d_bwd_weight_fp8", ctypes.byref(d), x8.data_ptr(), xdq.data_ptr(), dy8.data_ptr(), dydq.data_ptr(),
           slab.data_ptr(), bslab.data_ptr(), L.stream())
    dw = torch.empty(d.cout, d.cin, 3, 3, device="cuda")
    db = torch.empty(d.cout, device="cuda")
    L.call("fv_conv2d_wgrad_fp8_reduce", ctypes.byref(d), slab.data_ptr(), bslab.data_ptr(), dw.data_ptr(), db.data_ptr(),
           L.stream())
    torch.cuda.synchronize()
    return dw, db


class Diag:
    def __init__(self, m):
        self.names = {id(mod): n for n, mod in m.named_modules()}
        self.i = 0

    def __call__(self, kind, cs, **t):
        if kind != "wgrad" or t.get("q8") is None:
            return
        torch.cuda.synchronize()
        x8, xdq, dy8, dydq = t["q8"]
        d = cs.d
        N, H, W = d.n, d.h, d.w
        dw, db = t["dw"].clone(), (t["db"].clone() if t.get("db") is not None else None)
        xq = (x8.view(torch.float8_e4m3fn).float().view(N, H, W, d.cin).permute(0, 3, 1, 2) * xdq).double().cpu()
        dyq = (dy8.view(torch.float8_e4m3fn).float().view(N, H, W, d.cout).permute(0, 3, 1, 2) * dydq).double().cpu()
        rw = torch.nn.grad.conv2d_weight(xq, (d.cout, d.cin, 3, 3), dyq, padding=1)
        rb = dyq.sum((0, 2, 3))
        dw2, db2 = run_wg(d, x8, xdq, dy8, dydq)
        x8c, dy8c = x8.clone(), dy8.clone()
        dw3, db3 = run_wg(d, x8c, xdq.clone(), dy8c, dydq.clone())
        xb, dyb = x8.view(torch.uint8), dy8.view(torch.uint8)
        stats = {
            "x_zero": (xb & 0x7F).eq(0).float().mean().item(), "x_sub": ((xb & 0x78).eq(0) & (xb & 0x7).ne(0)).float().mean().item(),
            "dy_zero": (dyb & 0x7F).eq(0).float().mean().item(), "dy_sub": ((dyb & 0x78).eq(0) & (dyb & 0x7).ne(0)).float().mean().item(),
            "x_sat": (xb & 0x7F).eq(0x7E).float().mean().item(), "dy_sat": (dyb & 0x7F).eq(0x7E).float().mean().item(),
            "x_nan": (xb & 0x7F).eq(0x7F).float().mean().item(), "dy_nan": (dyb & 0x7F).eq(0x7F).float().mean().item(),
            "xdq": xdq.item(), "dydq": dydq.item(), "x8_numel": x8.numel(), "dy8_numel": dy8.numel(),
            "x_shape": tuple(t["x"].shape), "dy_shape": tuple(t["dy"].shape),
        }
        print(f"[{self.i}] {self.names.get(id(cs.conv), '?')}  step vs ref {rel(dw, rw):.2e} / bias {rel(db, rb) if db is not None else 0:.2e}"
              f" | rerun vs ref {rel(dw2, rw):.2e} / {rel(db2, rb):.2e} | copies vs ref {rel(dw3, rw):.2e} / {rel(db3, rb):.2e}"
              f" | step vs rerun {rel(dw, dw2):.2e}\n    {stats}", flush=True)
        self.i += 1


def main():
    torch.manual_seed(0)
    cfg = fv.FaceVAEConfig()
    m = fv.FaceVAE(cfg).cuda().train().set_compute_dtype(torch.float8_e4m3fn)
    x = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(1234)).cuda()
    eps = torch.randn(B, 256, 64, 64, generator=torch.Generator().manual_seed(1235)).cuda()
    ops.CHECK = Diag(m)
    try:
        y, mu, ls = m(x, eps)
        (cfg.w_R * fv.ReconLoss()((x, y)) + cfg.w_K * fv.KLDivergenceLoss()((mu, ls))).backward()
    finally:
        ops.CHECK = None
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
