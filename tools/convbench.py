"""Per-layer conv kernel timing at the FaceVAE shapes (256x256, B=32 by default).

    python tools/convbench.py [--batch 32] [--res 256] [--iters 20] [--only fwd,dgrad,wgrad] [--layers res,up2]

Times fv_conv2d_fwd / fv_conv2d_bwd_data / fv_conv2d_bwd_weight(+reduce) with HIP events on
the launch stream and prints us/launch and TFLOP/s (algorithmic, reference formulation).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import fvamd  # noqa: E402,F401
from facevae_amd import _lib as L  # noqa: E402
from facevae_amd import ops  # noqa: E402

CL = torch.channels_last


def layers(H):
    q, e = H // 4, H // 2
    # name, k, cin, cout, out H, ups
    return [
        ("in7", 7, 3, 64, H, False),
        ("down1", 3, 64, 128, H, False),
        ("down2", 3, 128, 256, e, False),
        ("mid1x1", 1, 256, 512, q, False),
        ("gin", 3, 256, 256, q, False),
        ("gmid1x1", 1, 256, 256, q, False),
        ("res", 3, 256, 256, q, False),
        ("up1", 3, 256, 128, e, True),
        ("up2", 3, 128, 64, H, True),
        ("out7", 7, 64, 3, H, False),
    ]


def timeit(fn, iters):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def diag_summary():
    """Per-wave clock stamps of the last halo-3x3 forward launch (diagnostic library):
    prologue (entry -> first barrier), main loop (of which: waits + barriers, the post-barrier
    issue block), epilogue, in shader cycles; the in-kernel clock from s_memtime / s_memrealtime
    (100 MHz) and the launch span."""
    n = 4096 * 8 * 8
    buf = (ctypes.c_ulonglong * n)()
    lib = L.load()
    lib.fv_diag_read.restype = ctypes.c_int
    if lib.fv_diag_read(buf, n) != 0:
        return None
    lib.fv_diag_clear()
    import numpy as np
    t = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    t = t[t[:, 0] != 0]
    if len(t) == 0:
        return None
    pro, loop, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    r0, r3 = t[:, 6], t[:, 7] & 0xffffffff
    r3 = r0 - (r0 & 0xffffffff) + r3 + np.where(r3 < (r0 & 0xffffffff), 1 << 32, 0)
    clk = (t[:, 3] - t[:, 0]) / np.maximum(r3 - r0, 1) * 0.1          # GHz
    span_us = (r3.max() - r0.min()) / 100.0
    starts = np.sort(np.unique(r0))
    out = {"waves": int(len(t)), "prologue": int(pro.mean()), "loop": int(loop.mean()), "loop_wait": int(t[:, 4].mean()),
           "loop_issue": int(t[:, 5].mean()), "epilogue": int(epi.mean()), "clock_ghz": round(float(np.median(clk)), 3),
           "span_us": round(float(span_us), 1),
           "wave_life_us": round(float(np.median(r3 - r0)) / 100.0, 1),
           "start_spread_us": round(float((starts[-1] - starts[0]) / 100.0), 1)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="fwd,dgrad,wgrad")
    ap.add_argument("--layers", default="")
    ap.add_argument("--dtype", default="bf16", help="bf16 | fp32 | fp8 (fp8 rows added for eligible layers)")
    ap.add_argument("--diag", action="store_true",
                    help="load the diagnostic library (build.py --diag) and print the in-kernel clock stamps "
                         "of the halo 3x3 forward after each layer's forward timing")
    ap.add_argument("--lib", default="", help="another build of libfacevae.so (A/B of two builds on one box)")
    a = ap.parse_args()
    if a.diag:
        L.LIB_PATH = os.path.join(ROOT, "face-vae_amd", "csrc", "build_diag", "libfacevae_diag.so")
    elif a.lib:
        L.LIB_PATH = os.path.abspath(a.lib)
    fp8 = a.dtype == "fp8"
    dtype = torch.bfloat16 if a.dtype in ("bf16", "fp8") else torch.float32
    kinds = a.only.split(",")
    sel = set(a.layers.split(",")) if a.layers else None
    B = a.batch
    out = []
    for name, k, cin, cout, H, ups in layers(a.res):
        if sel and name not in sel:
            continue
        Hi = H // 2 if ups else H
        cp = ops.pad_pow2(cin)
        x = torch.randn(B, cp, Hi, Hi, device="cuda").to(dtype).contiguous(memory_format=CL)
        d = ops.desc(dtype, B, H, H, cp, cin, cout, cout, k, ups)
        psc = psh = None
        w = (torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).contiguous()
        wk = torch.empty(L.query("fv_conv_wk_elems", ctypes.byref(d)), dtype=dtype, device="cuda")
        wt = torch.empty(L.query("fv_conv_wt_elems", ctypes.byref(d)), dtype=dtype, device="cuda")
        L.call("fv_conv_weight_prep", ctypes.byref(d), w.data_ptr(), None, wk.data_ptr(), wt.data_ptr(), L.stream())
        nchw = cout % 8 != 0
        ldd = ops.pad_pow2(cout) if nchw else cout
        if nchw:
            d.out_nchw_f32 = 1
            y = torch.empty(B, cout, H, H, device="cuda")
        else:
            y = torch.empty(B, cout, H, H, dtype=dtype, device="cuda", memory_format=CL)
        nb = L.query("fv_conv2d_stats_blocks", ctypes.byref(d))
        part = torch.empty(nb * 2 * cout, device="cuda")
        flop = 2.0 * B * H * H * cout * cin * k * k
        row = {"layer": name, "k": k, "cin": cin, "cout": cout, "H": H, "ups": ups, "gflop": flop / 1e9,
               "pro": psc is not None}
        if fp8 and L.query("fv_conv2d_fp8_supported", ctypes.byref(d)):
            # fp8 operands (quantized once, outside the timed region) for fwd and dgrad
            ws = torch.empty(L.query("fv_fp8_ws_bytes") // 4, device="cuda")
            x8 = torch.empty(x.numel(), dtype=torch.uint8, device="cuda")
            xdq, wdq, dydq = (torch.empty(1, device="cuda") for _ in range(3))
            L.call("fv_quantize_fp8", L.dtype_code(dtype), x.data_ptr(), x.numel(), x8.data_ptr(), xdq.data_ptr(),
                   ws.data_ptr(), L.stream())
            wk8 = torch.empty(L.query("fv_conv_fp8_wk_bytes", ctypes.byref(d)), dtype=torch.uint8, device="cuda")
            wt8 = torch.empty(L.query("fv_conv_fp8_wt_bytes", ctypes.byref(d)), dtype=torch.uint8, device="cuda")
            L.call("fv_conv_weight_prep_fp8", ctypes.byref(d), w.data_ptr(), None, wk8.data_ptr(), wt8.data_ptr(),
                   wdq.data_ptr(), ws.data_ptr(), L.stream())
            dyf = (torch.randn(B, cout, H, H, device="cuda") * 0.1).to(dtype).contiguous(memory_format=CL)
            dy8 = torch.empty(dyf.numel(), dtype=torch.uint8, device="cuda")
            L.call("fv_quantize_fp8", L.dtype_code(dtype), dyf.data_ptr(), dyf.numel(), dy8.data_ptr(),
                   dydq.data_ptr(), ws.data_ptr(), L.stream())
            if "fwd" in kinds:
                us = timeit(lambda: L.call("fv_conv2d_fwd_fp8", ctypes.byref(d), x8.data_ptr(), xdq.data_ptr(),
                                           wk8.data_ptr(), wdq.data_ptr(), None, None, y.data_ptr(), part.data_ptr(),
                                           L.stream()), a.iters)
                row["fp8_fwd_us"], row["fp8_fwd_tf"] = round(us, 1), round(flop / us / 1e6, 1)
                us = timeit(lambda: L.call("fv_quantize_fp8", L.dtype_code(dtype), x.data_ptr(), x.numel(),
                                           x8.data_ptr(), xdq.data_ptr(), ws.data_ptr(), L.stream()), a.iters)
                row["fp8_quant_us"] = round(us, 1)
            if "wgrad" in kinds and L.query("fv_conv2d_wgrad_fp8_supported", ctypes.byref(d)):
                slab8 = torch.empty(L.query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), device="cuda")
                bslab8 = torch.empty(L.query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), device="cuda")
                us = timeit(lambda: L.call("fv_conv2d_bwd_weight_fp8", ctypes.byref(d), x8.data_ptr(), xdq.data_ptr(),
                                           dy8.data_ptr(), dydq.data_ptr(), slab8.data_ptr(), bslab8.data_ptr(),
                                           L.stream()), a.iters)
                row["fp8_wgrad_us"], row["fp8_wgrad_tf"] = round(us, 1), round(flop / us / 1e6, 1)
            if "dgrad" in kinds:
                dxf = torch.empty(B, cp, H, H, dtype=dtype, device="cuda", memory_format=CL)
                us = timeit(lambda: L.call("fv_conv2d_bwd_data_fp8", ctypes.byref(d), dy8.data_ptr(), dydq.data_ptr(),
                                           wt8.data_ptr(), wdq.data_ptr(), dxf.data_ptr(), L.stream()), a.iters)
                row["fp8_dgrad_us"], row["fp8_dgrad_tf"] = round(us, 1), round(flop / us / 1e6, 1)
        if "fwd" in kinds:
            if a.diag:
                L.load().fv_diag_clear()
            us = timeit(lambda: L.call("fv_conv2d_fwd", ctypes.byref(d), x.data_ptr(), wk.data_ptr(), None, L.ptr(psc),
                                       L.ptr(psh), None, y.data_ptr(), None if nchw else part.data_ptr(), L.stream()),
                        a.iters)
            row["fwd_us"], row["fwd_tf"] = round(us, 1), round(flop / us / 1e6, 1)
            if a.diag:
                row["diag_fwd"] = diag_summary()
        dy = (torch.randn(B, ldd, H, H, device="cuda") * 0.1).to(dtype).contiguous(memory_format=CL)
        if "dgrad" in kinds and name != "in7" and psc is None:
            dx = torch.empty(B, cp, H, H, dtype=dtype, device="cuda", memory_format=CL)
            if a.diag:
                L.load().fv_diag_clear()
            us = timeit(lambda: L.call("fv_conv2d_bwd_data", ctypes.byref(d), dy.data_ptr(), ldd, wt.data_ptr(),
                                       dx.data_ptr(), L.stream()), a.iters)
            row["dgrad_us"], row["dgrad_tf"] = round(us, 1), round(flop / us / 1e6, 1)
            if a.diag:
                row["diag_dgrad"] = diag_summary()
        if "wgrad" in kinds:
            slab = torch.empty(L.query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), device="cuda")
            bslab = torch.empty(L.query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), device="cuda")
            dw = torch.empty_like(w)
            db = torch.empty(cout, device="cuda")
            us = timeit(lambda: L.call("fv_conv2d_bwd_weight", ctypes.byref(d), x.data_ptr(), L.ptr(psc), L.ptr(psh),
                                       dy.data_ptr(), ldd, slab.data_ptr(), bslab.data_ptr(), L.stream()), a.iters)
            us2 = timeit(lambda: L.call("fv_conv2d_wgrad_reduce", ctypes.byref(d), slab.data_ptr(), bslab.data_ptr(),
                                        dw.data_ptr(), db.data_ptr(), L.stream()), a.iters)
            row["wgrad_us"], row["wgrad_tf"], row["wred_us"] = round(us, 1), round(flop / us / 1e6, 1), round(us2, 1)
        out.append(row)
        print(json.dumps(row), flush=True)
    tot = {k: round(sum(r.get(k, 0) for r in out), 1) for k in ("fwd_us", "dgrad_us", "wgrad_us", "wred_us")}
    print(json.dumps({"total": tot}))


if __name__ == "__main__":
    main()
