"""fp8 (OCP e4m3) conv path (BASELINE config C5): conversion, the scaled-MFMA fragment layout,
and the fp8 forward / data-gradient conv kernels against torch fp32 on the dequantized
operands (the products of two e4m3 values are exact in fp32, so kernel and reference differ
only by fp32 summation order and the bf16 rounding of the output)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

import facevae_amd as fv  # noqa: E402
from facevae_amd import _lib as L  # noqa: E402
from facevae_amd import ops  # noqa: E402

CL = torch.channels_last


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def quant(x):
    """library quantization of a contiguous bf16/f32 tensor -> (uint8 tensor, dq tensor)"""
    y = torch.empty(x.numel(), dtype=torch.uint8, device="cuda")
    dq = torch.empty(1, device="cuda")
    ws = torch.empty(L.query("fv_fp8_ws_bytes") // 4, device="cuda")
    L.call("fv_quantize_fp8", L.dtype_code(x.dtype), x.data_ptr(), x.numel(), y.data_ptr(), dq.data_ptr(),
           ws.data_ptr(), L.stream())
    return y, dq


def deq(y8, dq, shape):
    return y8.view(torch.float8_e4m3fn).float().view(shape) * dq


def test_quantize_matches_torch_e4m3():
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(100003, generator=g) * 3.7).cuda()
    x[17] = 0.0
    y8, dq = quant(x)
    torch.cuda.synchronize()
    s = 1.0 / dq.item()
    amax = x.abs().max().item()
    assert s * amax <= 448 and s * amax > 224 and s == 2.0 ** round(torch.log2(torch.tensor(s)).item())
    ref = (x * s).to(torch.float8_e4m3fn)            # torch: OCP e4m3fn, round to nearest even
    assert torch.equal(y8.view(torch.float8_e4m3fn).view(torch.uint8), ref.view(torch.uint8))


def test_fp8_mfma_fragment_layout():
    g = torch.Generator().manual_seed(2)
    a = torch.randn(16, 128, generator=g).to(torch.float8_e4m3fn)
    b = torch.randn(16, 128, generator=g).to(torch.float8_e4m3fn)
    c = torch.empty(16, 16, device="cuda")
    ac, bc = a.view(torch.uint8).cuda(), b.view(torch.uint8).cuda()
    L.call("fv_fp8_mfma_probe", ac.data_ptr(), bc.data_ptr(), c.data_ptr(), L.stream())
    torch.cuda.synchronize()
    ref = a.double() @ b.double().t()
    assert rel(c, ref) < 1e-4      # (the 128-term sum inside the scaled MFMA: ~1e-5 relative)


CASES = [(256, 256, 8, 64, 2), (128, 256, 4, 128, 2), (256, 128, 12, 64, 1), (256, 256, 64, 64, 32)]


@pytest.mark.parametrize("case", CASES)
def test_conv_fp8_fwd_and_dgrad(case, monkeypatch):
    cin, cout, H, W, N = case
    g = torch.Generator().manual_seed(3 + cin + H)
    x = torch.randn(N, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    b = torch.randn(cout, generator=g)
    dy = torch.randn(N, cout, H, W, generator=g)
    xb = x.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    d = ops.desc(torch.bfloat16, N, H, W, cin, cin, cout, cout, 3)
    assert L.query("fv_conv2d_fp8_supported", ctypes.byref(d))
    x8, xdq = quant(xb)
    wk = torch.empty(L.query("fv_conv_fp8_wk_bytes", ctypes.byref(d)), dtype=torch.uint8, device="cuda")
    wt = torch.empty(L.query("fv_conv_fp8_wt_bytes", ctypes.byref(d)), dtype=torch.uint8, device="cuda")
    wdq = torch.empty(1, device="cuda")
    ws = torch.empty(L.query("fv_fp8_ws_bytes") // 4, device="cuda")
    wc = w.cuda().contiguous()
    L.call("fv_conv_weight_prep_fp8", ctypes.byref(d), wc.data_ptr(), None, wk.data_ptr(), wt.data_ptr(),
           wdq.data_ptr(), ws.data_ptr(), L.stream())
    y = torch.empty(N, cout, H, W, dtype=torch.bfloat16, device="cuda", memory_format=CL)
    nb = L.query("fv_conv2d_stats_blocks", ctypes.byref(d))
    part = torch.empty(nb * 2 * cout, device="cuda")
    L.call("fv_conv2d_fwd_fp8", ctypes.byref(d), x8.data_ptr(), xdq.data_ptr(), wk.data_ptr(), wdq.data_ptr(),
           b.cuda().data_ptr(), None, y.data_ptr(), None, L.stream())
    # data gradient
    dyb = dy.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    dy8, dydq = quant(dyb)
    dx = torch.empty(N, cin, H, W, dtype=torch.bfloat16, device="cuda", memory_format=CL)
    L.call("fv_conv2d_bwd_data_fp8", ctypes.byref(d), dy8.data_ptr(), dydq.data_ptr(), wt.data_ptr(),
           wdq.data_ptr(), dx.data_ptr(), L.stream())
    torch.cuda.synchronize()
    # the SIMD-partner schedules (FV_RES_SCHED, conv3_halo_fp8 SCH) only reorder instructions
    for sched in (0, 1, 2, 3):
        monkeypatch.setenv("FV_RES_SCHED", str(sched))
        y2, dx2 = torch.empty_like(y), torch.empty_like(dx)
        L.call("fv_conv2d_fwd_fp8", ctypes.byref(d), x8.data_ptr(), xdq.data_ptr(), wk.data_ptr(), wdq.data_ptr(),
               b.cuda().data_ptr(), None, y2.data_ptr(), None, L.stream())
        L.call("fv_conv2d_bwd_data_fp8", ctypes.byref(d), dy8.data_ptr(), dydq.data_ptr(), wt.data_ptr(),
               wdq.data_ptr(), dx2.data_ptr(), L.stream())
        torch.cuda.synchronize()
        assert torch.equal(y2, y) and torch.equal(dx2, dx), f"schedule {sched} differs"
    monkeypatch.delenv("FV_RES_SCHED")
    # references on the dequantized fp8 operands (NHWC byte order -> NCHW)
    xq = deq(x8, xdq, (N, H, W, cin)).permute(0, 3, 1, 2)
    wq = deq(wk, wdq, (cout, 3, 3, cin)).permute(0, 3, 1, 2)
    ref = F.conv2d(xq.double().cpu(), wq.double().cpu(), b.double(), padding=1)
    dyq = deq(dy8, dydq, (N, H, W, cout)).permute(0, 3, 1, 2)
    refdx = torch.nn.grad.conv2d_input((N, cin, H, W), wq.double().cpu(), dyq.double().cpu(), padding=1)
    for out, r in ((y, ref), (dx, refdx)):
        dd = (out.double().cpu() - r).abs()
        bound = 2.0 ** -7 * r.abs() + 2e-3 * r.pow(2).mean().sqrt()
        assert (dd / bound).max().item() <= 1.0 and rel(out, r) < 5e-3
    # the fp8 rounding itself vs the unquantized fp32 conv (reported: ~2^-5 relative per operand)
    dev = rel(y, F.conv2d(x, w, b, padding=1))
    print(f"\n[fp8 conv {case}] output rel-L2 vs unquantized fp32 conv: {dev:.3e}")
    assert dev < 0.1


def test_delayed_scaling_site():
    """fv_quantize_fp8_site: the first call is exact (bytes and dq of fv_quantize_fp8); later
    calls quantize with the pow2 scale of the 16-deep amax history, saturating at +-448, and the
    consuming *_site conv moves each call's amax into the history."""
    N, C, H, W = 2, 128, 4, 64
    d = ops.desc(torch.bfloat16, N, H, W, C, C, C, C, 3)
    w = (torch.randn(C, C, 3, 3, generator=torch.Generator().manual_seed(7)) / (C * 9) ** 0.5).cuda()
    wk = torch.empty(L.query("fv_conv_fp8_wk_bytes", ctypes.byref(d)), dtype=torch.uint8, device="cuda")
    wdq = torch.empty(1, device="cuda")
    ws = torch.empty(L.query("fv_fp8_ws_bytes") // 4, device="cuda")
    L.call("fv_conv_weight_prep_fp8", ctypes.byref(d), w.data_ptr(), None, wk.data_ptr(), None, wdq.data_ptr(),
           ws.data_ptr(), L.stream())
    y = torch.empty(N, C, H, W, dtype=torch.bfloat16, device="cuda").contiguous(memory_format=CL)
    site = [torch.zeros(L.query("fv_fp8_site_bytes") // 4, dtype=torch.int32, device="cuda"), False]

    def conv(x8):
        L.call("fv_conv2d_fwd_fp8_site", ctypes.byref(d), x8.data_ptr(), site[0].data_ptr(), wk.data_ptr(),
               wdq.data_ptr(), None, None, y.data_ptr(), None, L.stream())

    g = torch.Generator().manual_seed(8)
    x1 = torch.randn(N, C, H, W, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    x2 = (x1.float() * 5.0).to(torch.bfloat16).contiguous(memory_format=CL)       # amax grows 5x
    q1, dq1 = ops.quantize_fp8_site(x1, site)
    e1, edq1 = quant(x1)
    torch.cuda.synchronize()
    assert torch.equal(q1, e1) and dq1.item() == edq1.item()
    conv(q1)
    q2, dq2 = ops.quantize_fp8_site(x2, site)        # delayed: x1's scale, x2 saturates
    torch.cuda.synchronize()
    s1 = 1.0 / edq1.item()
    assert dq2.item() == edq1.item()
    ref2 = (x2.float() * s1).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(q2, ref2.permute(0, 2, 3, 1).reshape(-1).view(torch.uint8))       # NHWC bytes
    conv(q2)
    q3, dq3 = ops.quantize_fp8_site(x2, site)        # the history now holds x2's amax
    e3, edq3 = quant(x2)
    torch.cuda.synchronize()
    assert dq3.item() == edq3.item() and torch.equal(q3, e3)


@pytest.mark.parametrize("addend", [False, True])
def test_bn_passes_write_the_fp8_operand(addend):
    """fv_bn_act_fwd_q8 / fv_bn_act_bwd_apply_q8: the bf16 output equals the plain BN pass, and
    the e4m3 copy, dq and the site's in-flight amax equal fv_quantize_fp8_site over that output
    on an identical copy of the site (delayed scale: the history is seeded with a smaller amax,
    so part of the output saturates)."""
    g = torch.Generator().manual_seed(21)
    N, C, H, W = 2, 256, 8, 64
    y = (torch.randn(N, C, H, W, generator=g) * 2).to(torch.bfloat16).cuda().contiguous(memory_format=CL)
    dout = torch.randn(N, C, H, W, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=CL)
    add = torch.randn(N, C, H, W, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=CL) if addend \
        else None
    bn = torch.nn.BatchNorm2d(C).cuda()                    # affine parameter holder
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
    r = ops._bn_result(C, y.device, N * H * W)
    r.mean.copy_(torch.randn(C, generator=g).cuda() * 0.1)
    r.invstd.copy_(torch.rand(C, generator=g).cuda() + 0.5)
    r.scale.copy_(bn.weight.detach() * r.invstd)
    r.shift.copy_(bn.bias.detach() - r.mean * r.scale)

    def seeded_site():
        s = [torch.zeros(L.query("fv_fp8_site_bytes") // 4, dtype=torch.int32, device="cuda"), True]
        s[0][:16] = torch.tensor([1.5], dtype=torch.float32).view(torch.int32).item()
        return s

    # forward pass
    sa, sb = seeded_site(), seeded_site()
    out, q = ops.bn_act_forward_q8(y, r, 0.0, bn, sa)
    ref = ops.bn_act_forward(y, r, 0.0, False, bn)
    rq, rdq = ops.quantize_fp8_site(ref, sb)
    torch.cuda.synchronize()
    assert q is not None and torch.equal(out, ref)
    assert torch.equal(q[0], rq) and q[1].item() == rdq.item() and torch.equal(sa[0], sb[0])
    # backward apply
    sa, sb = seeded_site(), seeded_site()
    dx, _, _, q = ops.bn_act_backward(dout, y, bn, r, 0.0, False, None, addend=add, q8=sa)
    # the same BN backward (same reduce, same k) without the site, then the separate quantize
    dx2, _, _ = ops.bn_act_backward(dout, y, bn, r, 0.0, False, None, addend=add)
    rq, rdq = ops.quantize_fp8_site(dx2, sb)
    torch.cuda.synchronize()
    assert q is not None and torch.equal(dx, dx2)
    assert torch.equal(q[0], rq) and q[1].item() == rdq.item() and torch.equal(sa[0], sb[0])
    # only8: the e4m3 copy alone, bit-identical, the bf16 output a 0-element placeholder
    sa, sb = seeded_site(), seeded_site()
    out, q = ops.bn_act_forward_q8(y, r, 0.0, bn, sa, only8=True)
    _, rq = ops.bn_act_forward_q8(y, r, 0.0, bn, sb)
    torch.cuda.synchronize()
    assert out.numel() == 0 and out.dtype == y.dtype
    assert torch.equal(q[0], rq[0]) and q[1].item() == rq[1].item() and torch.equal(sa[0], sb[0])
    sa, sb = seeded_site(), seeded_site()
    dx, _, _, q = ops.bn_act_backward(dout, y, bn, r, 0.0, False, None, addend=add, q8=sa, only8=True)
    _, _, _, rq = ops.bn_act_backward(dout, y, bn, r, 0.0, False, None, addend=add, q8=sb)
    torch.cuda.synchronize()
    assert dx.numel() == 0 and dx.dtype == y.dtype
    assert torch.equal(q[0], rq[0]) and q[1].item() == rq[1].item() and torch.equal(sa[0], sb[0])


def test_resblock_fp8_only8_matches_bf16_copies():
    """q8_only: the ResBlock's fp8 BN passes (a1, a2 forward; dt1 backward) write the e4m3 copy
    alone when the consuming conv's forward, dgrad and wgrad all run on e4m3.  Output and every
    gradient equal the run that also writes the bf16 tensors, and the placeholders are taken."""
    from facevae_amd.modules import ResBlock2D
    N, C, H, W = 2, 256, 8, 64
    g = torch.Generator().manual_seed(41)
    x0 = torch.randn(N, C, H, W, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    g1 = torch.randn(N, C, H, W, generator=g).cuda()
    torch.manual_seed(7)
    blk = ResBlock2D(C, True).cuda().train().set_compute_dtype(torch.float8_e4m3fn)
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    seen = []
    orig = ops.bn_act_forward_q8

    def spy(*a, **k):
        r = orig(*a, **k)
        seen.append(r[0].numel() == 0)
        return r

    def run(only8):
        blk.load_state_dict(sd)
        for m in (blk, blk.conv1, blk.conv2):
            m.__dict__.pop("_fv_fp8_sites", None)
            m.__dict__.pop("_fv_fp8_pending", None)
        ops._Q8_ONLY = only8
        ops.bn_act_forward_q8 = spy
        seen.clear()
        try:
            for _ in range(2):                        # step 1 seeds the delayed-scaling sites
                x = x0.clone().requires_grad_(True)
                for p in blk.parameters():
                    p.grad = None
                out = blk(x)
                (out.float() * g1).sum().backward()
            torch.cuda.synchronize()
            return out.detach().clone(), x.grad.clone(), [p.grad.clone() for p in blk.parameters()], list(seen)
        finally:
            ops._Q8_ONLY = True
            ops.bn_act_forward_q8 = orig

    o_on, dx_on, gr_on, seen_on = run(True)
    o_off, dx_off, gr_off, seen_off = run(False)
    assert torch.equal(o_on, o_off) and torch.equal(dx_on, dx_off)
    for a, b in zip(gr_on, gr_off):
        assert torch.equal(a, b)
    assert seen_on[-2:] == [True, True] and not any(seen_off)


def test_resblock_fp8_store_pass_statistics():
    """fp8 ResBlock conv2 with the store-pass reduction in the e4m3 conv's epilogue
    (fv_conv2d_fwd_fp8_site_sr): the output equals the run without it bit for bit, and the
    records it hands to the next ResBlock's bn1 sum to the statistics of the stored output."""
    from facevae_amd.modules import ResBlock2D
    N, C, H, W = 2, 256, 8, 64
    g = torch.Generator().manual_seed(43)
    x0 = torch.randn(N, C, H, W, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    torch.manual_seed(9)
    blk = ResBlock2D(C, True).cuda().train().set_compute_dtype(torch.float8_e4m3fn)
    sd = {k: v.clone() for k, v in blk.state_dict().items()}

    def run(sr):
        blk.load_state_dict(sd)
        for m in (blk, blk.conv1, blk.conv2):
            m.__dict__.pop("_fv_fp8_sites", None)
            m.__dict__.pop("_fv_fp8_pending", None)
        ops.FP8_SR = sr
        try:
            for _ in range(2):                        # step 1 seeds the delayed-scaling sites
                out = blk(x0.clone())
            torch.cuda.synchronize()
            return out.detach().clone(), getattr(out, "_fv_bnrec", None)
        finally:
            ops.FP8_SR = True

    o_on, rec = run(True)
    o_off, rec_off = run(False)
    assert torch.equal(o_on, o_off)
    assert rec is not None and rec_off is None
    part, nrec, bp = rec[0], rec[1], rec[2]
    assert nrec * bp == N * H * W
    r = part.view(nrec, 2, C).double().sum(0).cpu()
    y = o_on.double().permute(1, 0, 2, 3).reshape(C, -1).cpu()
    assert ((r[0] - y.sum(1)).abs() / y.abs().sum(1)).max() < 1e-5
    assert ((r[1] - (y * y).sum(1)).abs() / (y * y).sum(1)).max() < 1e-5


@pytest.mark.parametrize("two_consumers", [False, True])
def test_resblock_fp8_handoff_checks_the_gradient_tensor(two_consumers):
    """the next ResBlock's bn1 backward leaves an e4m3 copy of its output for this
    block's conv2 data gradient.  With a second consumer of the block output autograd adds the
    other gradient into that tensor (in place: same pointer, new version) before conv2's backward
    runs, so the copy is stale and must be rejected.  Gradients with the hand-off on equal those
    with it off (every dy quantized by its conv), and the hand-off is still taken when the output
    has one consumer."""
    from facevae_amd.modules import ResBlock2D
    N, C, H, W = 2, 256, 8, 64
    g = torch.Generator().manual_seed(31)
    x0 = torch.randn(N, C, H, W, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    g1 = torch.randn(N, C, H, W, generator=g).cuda()
    g2 = torch.randn(N, C, H, W, generator=g).cuda()
    torch.manual_seed(5)
    r1, r2 = ResBlock2D(C, True), ResBlock2D(C, True)
    r1, r2 = r1.cuda().train().set_compute_dtype(torch.float8_e4m3fn), r2.cuda().train().set_compute_dtype(
        torch.float8_e4m3fn)
    state = [{k: v.clone() for k, v in m.state_dict().items()} for m in (r1, r2)]
    calls = []
    orig = ops.quantize_fp8_site

    def counting(t, site):
        calls.append(t.shape)
        return orig(t, site)

    def run(handoff):
        for m, sd in zip((r1, r2), state):
            m.load_state_dict(sd)
            m.__dict__.pop("_fv_fp8_sites", None)
            for c in (m.conv1, m.conv2):
                c.__dict__.pop("_fv_fp8_sites", None)
                c.__dict__.pop("_fv_fp8_pending", None)
        ops._FP8_HANDOFF = handoff
        try:
            out = None
            for it in range(2):                       # step 1 seeds the delayed-scaling sites
                x = x0.clone().requires_grad_(True)
                for p in list(r1.parameters()) + list(r2.parameters()):
                    p.grad = None
                h = r1(x)
                out = r2(h)
                loss = (out.float() * g1).sum()
                if two_consumers:
                    loss = loss + (h.float() * g2).sum()
                calls.clear()
                ops.quantize_fp8_site = counting
                try:
                    loss.backward()
                finally:
                    ops.quantize_fp8_site = orig
            torch.cuda.synchronize()
            return x.grad.clone(), [p.grad.clone() for p in r1.parameters()], len(calls)
        finally:
            ops._FP8_HANDOFF = True

    dx_on, gr_on, nq_on = run(True)
    dx_off, gr_off, nq_off = run(False)
    assert torch.equal(dx_on, dx_off)
    for a, b in zip(gr_on, gr_off):
        assert torch.equal(a, b)
    if two_consumers:
        assert nq_on == nq_off            # the stale copy is rejected: dy quantized again
    else:
        assert nq_on == nq_off - 1        # the copy is taken: one quantize pass fewer


def test_tr8_transposed_read_lane_mapping():
    """ds_read_b64_tr_b8 (gfx950): within each 16-lane group, lane li supplies the address of an
    8-byte segment -- row li >> 1, columns 8 (li & 1) .. +7 -- of an 8 x 16 byte block, and lane li
    receives COLUMN li of the block (its 8 rows, row 0 in the lowest byte): the 8-bit form of the
    ds_read_b64_tr_b16 transpose the bf16 weight gradients use.  Pinned here before the fp8
    weight gradient relies on it."""
    ROWB = 16
    lanes = torch.arange(64)
    li, g = lanes & 15, lanes >> 4
    addr = (g * 256 + (li >> 1) * ROWB + (li & 1) * 8).to(torch.int32).cuda()
    out = torch.empty(128, dtype=torch.int32, device="cuda")
    L.call("fv_tr8_probe", addr.data_ptr(), out.data_ptr(), L.stream())
    torch.cuda.synchronize()
    got = out.cpu().view(64, 2).contiguous().view(torch.uint8).view(64, 8)
    exp = torch.empty(64, 8, dtype=torch.uint8)
    for lane in range(64):
        for r in range(8):
            exp[lane, r] = (int(g[lane]) * 256 + r * ROWB + int(li[lane])) & 255
    print("\n[tr_b8] group 0 received (lane: bytes):\n" + "\n".join(
        f"  {i:2d}: {got[i].tolist()}" for i in range(16)))
    assert torch.equal(got, exp)


def test_fp8_mfma_subnormal_operands():
    """e4m3 subnormals (|v| < 2^-6) enter the scaled MFMA as their exact values (no flush)."""
    g = torch.Generator().manual_seed(5)
    a = (torch.randn(16, 128, generator=g) * 2.0 ** -8).to(torch.float8_e4m3fn)
    b = torch.randn(16, 128, generator=g).to(torch.float8_e4m3fn)
    frac = (a.view(torch.uint8) & 0x78).eq(0).float().mean().item()
    assert frac > 0.5                                # mostly subnormal (exponent field 0)
    c = torch.empty(16, 16, device="cuda")
    ac, bc = a.view(torch.uint8).cuda(), b.view(torch.uint8).cuda()      # (held: distinct buffers)
    L.call("fv_fp8_mfma_probe", ac.data_ptr(), bc.data_ptr(), c.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert rel(c, a.double() @ b.double().t()) < 1e-4


def test_fp8_mfma_accumulation_groups():
    """The scaled fp8 MFMA does not add its 128 products exactly: within a group of 8 products
    (k = 8 j .. 8 j + 7) the terms are aligned to the group's largest and truncated ~13 bits
    below it (measured r4: 448 + 127 x 2^-9 -> 448.234375, the 7 small terms sharing the big
    one's group are lost; 64 + 127 x 2^-6 is exact).  The fp8 weight-gradient gates assume
    |error| <= 8 x 2^-13 x (the largest product of a group) per group, i.e. <= 2^-10 sum|terms|."""
    ones = torch.ones(16, 128)
    cases = []
    for big in (448.0, 64.0, 8.0):
        for small in (2.0 ** -9, 2.0 ** -6, 0.125):
            a = torch.full((16, 128), small)
            a[:, 0] = big
            cases.append(a)
    a = torch.full((16, 128), 2.0 ** -7)
    a[:, 0], a[:, 1] = 448.0, -448.0
    cases.append(a)
    g = torch.Generator().manual_seed(7)
    cases.append(torch.randn(16, 128, generator=g) ** 3 * 4)
    lost = []
    for a in cases:
        a8 = a.to(torch.float8_e4m3fn)
        ac, bc = a8.view(torch.uint8).cuda(), ones.to(torch.float8_e4m3fn).view(torch.uint8).cuda()
        c = torch.empty(16, 16, device="cuda")
        L.call("fv_fp8_mfma_probe", ac.data_ptr(), bc.data_ptr(), c.data_ptr(), L.stream())
        torch.cuda.synchronize()
        t = a8.double()
        exact = t.sum(1)
        bound = 8 * 2.0 ** -13 * t.abs().view(16, 16, 8).amax(2).sum(1)
        err = (c[:, 0].double().cpu() - exact).abs()
        assert (err <= bound).all(), (err, bound)
        lost.append(err.max().item())
    print(f"\n[fp8 MFMA] largest lost amount per probe: {lost}")
    assert lost[0] == 7 * 2.0 ** -9        # the group-of-8 truncation this gate models is present


WG_CASES = [("randn", 8), ("centered", 8), ("heavy", 8), ("centered", 64), ("heavy_centered", 64)]


@pytest.mark.parametrize("kind,N", WG_CASES)
def test_conv_fp8_wgrad(kind, N):
    """fv_conv2d_bwd_weight_fp8 at the ResBlock shape (256 -> 256, 64x64) against float64 on the
    dequantized operands, elementwise at 2^-10 of the sum of |terms| (the fp8 MFMA's group-of-8
    truncation, test_fp8_mfma_accumulation_groups; fp32 across groups).  centered: dy with its
    per-channel pixel mean removed -- the gradient a conv followed by a BN receives (the bias
    sum cancels); heavy: x = randn^3, many subnormals."""
    cin = cout = 256
    H = W = 64
    g = torch.Generator().manual_seed(11 + N)
    x = torch.randn(N, cin, H, W, generator=g)
    dy = torch.randn(N, cout, H, W, generator=g)
    if kind == "heavy":
        x = x ** 3
    if kind == "heavy_centered":                 # a BN-backward-like dy: heavy tails, zero pixel sums
        x = torch.relu(x)
        dy = dy ** 3
    if kind in ("centered", "heavy_centered"):
        dy = dy - dy.mean((0, 2, 3), keepdim=True)
    d = ops.desc(torch.bfloat16, N, H, W, cin, cin, cout, cout, 3)
    assert L.query("fv_conv2d_wgrad_fp8_supported", ctypes.byref(d))
    x8, xdq = quant(x.cuda().to(torch.bfloat16).contiguous(memory_format=CL))
    dy8, dydq = quant(dy.cuda().to(torch.bfloat16).contiguous(memory_format=CL))
    slab = torch.empty(L.query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), device="cuda")
    bslab = torch.empty(L.query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), device="cuda")
    L.call("fv_conv2d_bwd_weight_fp8", ctypes.byref(d), x8.data_ptr(), xdq.data_ptr(), dy8.data_ptr(),
           dydq.data_ptr(), slab.data_ptr(), bslab.data_ptr(), L.stream())
    dw = torch.empty(cout, cin, 3, 3, device="cuda")
    db = torch.empty(cout, device="cuda")
    L.call("fv_conv2d_wgrad_fp8_reduce", ctypes.byref(d), slab.data_ptr(), bslab.data_ptr(), dw.data_ptr(),
           db.data_ptr(), L.stream())
    torch.cuda.synchronize()
    xq = deq(x8, xdq, (N, H, W, cin)).permute(0, 3, 1, 2).double().cpu()
    dyq = deq(dy8, dydq, (N, H, W, cout)).permute(0, 3, 1, 2).double().cpu()
    rw = torch.nn.grad.conv2d_weight(xq, (cout, cin, 3, 3), dyq, padding=1)
    aw = torch.nn.grad.conv2d_weight(xq.abs(), (cout, cin, 3, 3), dyq.abs(), padding=1)
    rb, ab = dyq.sum((0, 2, 3)), dyq.abs().sum((0, 2, 3))
    ew = ((dw.double().cpu() - rw).abs() / (2.0 ** -10 * aw + 1e-30)).max().item()
    eb = ((db.double().cpu() - rb).abs() / (2.0 ** -10 * ab + 1e-30)).max().item()
    print(f"\n[fp8 wgrad {kind} N={N}] worst |d| / (2^-10 sum|terms|): weight {ew:.4f} bias {eb:.4f}; "
          f"rel-L2 weight {rel(dw, rw):.2e} bias {rel(db, rb):.2e}")
    assert ew <= 1.0 and eb <= 1.0


def test_fp8_weight_prep_batched_bit_identical(monkeypatch):
    """The per-step e4m3 weight quantization of every fp8 conv batched into two launches
    (ops.WPrepBatch -> fv_conv_weight_prep_fp8_multi) against the per-conv
    fv_conv_weight_prep_fp8 launches: three fp8 training steps of the FaceVAE at 256², B=2 give
    bit-identical parameters, losses and output."""
    cfg = fv.FaceVAEConfig()
    g = torch.Generator().manual_seed(5)
    x = torch.rand(2, 3, cfg.H, cfg.H, generator=g).cuda()
    eps = torch.randn(2, cfg.latent, cfg.latent_hw, cfg.latent_hw, generator=g).cuda()
    torch.manual_seed(0)
    init = {k: v.clone() for k, v in fv.FaceVAE(cfg).state_dict().items()}
    res, counts = [], []
    names = []
    orig_call = ops.call

    def spy(name, *a):
        names.append(name)
        return orig_call(name, *a)

    monkeypatch.setattr(ops, "call", spy)
    for batch in (False, True):
        monkeypatch.setattr(ops, "_WPREP_FP8_BATCH", batch)
        names.clear()
        m = fv.FaceVAE(cfg).cuda().train().set_compute_dtype(torch.float8_e4m3fn)
        m.load_state_dict(init)
        opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            y, mu, ls = m(x, eps)
            R, K = fv.ReconLoss()((x, y)), fv.KLDivergenceLoss()((mu, ls))
            (R + K).backward()
            opt.step()
        torch.cuda.synchronize()
        counts.append((names.count("fv_conv_weight_prep_fp8"), names.count("fv_conv_weight_prep_fp8_multi")))
        res.append((y.detach().float().cpu(), R.item(), K.item(),
                    {k: p.detach().cpu().clone() for k, p in m.named_parameters()}))
    # per-conv quantization in every step without batching; with it only in the first step (no
    # forward has recorded the descriptors yet), then one two-launch call per step
    (n1_off, nm_off), (n1_on, nm_on) = counts
    assert n1_off > 0 and nm_off == 0 and n1_on * 3 == n1_off and nm_on == 2, counts
    (y0, r0, k0, p0), (y1, r1, k1, p1) = res
    assert torch.equal(y0, y1) and r0 == r1 and k0 == k1
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k


def test_fp8_dq_view_survives_a_second_forward():
    """The fp8 weight gradient reads the forward's x scale (dq) as a view of the conv's
    delayed-scaling site (no copy per forward).  A second forward through the same block before
    the first one's backward re-quantizes the site with another scale (4x larger input): the
    first backward must still see ITS dq (ops._dq_snapshot copies it just before the site is
    re-quantized), so every gradient equals the run without the second forward, bit for bit."""
    from facevae_amd.modules import ResBlock2D
    N, C, H, W = 2, 256, 8, 64
    g = torch.Generator().manual_seed(47)
    x0 = torch.randn(N, C, H, W, generator=g).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    g1 = torch.randn(N, C, H, W, generator=g).cuda()
    torch.manual_seed(11)
    blk = ResBlock2D(C, False).cuda().train().set_compute_dtype(torch.float8_e4m3fn)
    sd = {k: v.clone() for k, v in blk.state_dict().items()}

    def site_dq():
        return blk.conv1.__dict__["_fv_fp8_sites"]["x"][0][18:19].view(torch.float32)

    def run(second):
        blk.load_state_dict(sd)
        for m in blk.modules():
            m.__dict__.pop("_fv_fp8_sites", None)
        x = x0.clone().requires_grad_(True)
        blk(x).float().mul(g1).sum().backward()     # step 1 seeds the sites
        for p in blk.parameters():
            p.grad = None
        x = x0.clone().requires_grad_(True)
        out = blk(x)
        dq_first = site_dq().clone()
        if second:
            # a spike survives BN's normalisation: the x sites' amax grows, and the second of
            # these forwards quantizes with the grown (delayed) scale
            x2 = x0.clone()
            x2[:, :, 0, 0] = 50.0
            for _ in range(2):
                blk(x2)
            assert not torch.equal(site_dq(), dq_first), "the test needs the site's dq to change"
        (out.float() * g1).sum().backward()
        torch.cuda.synchronize()
        return x.grad.clone(), [p.grad.clone() for p in blk.parameters()]

    dx_a, gr_a = run(False)
    dx_b, gr_b = run(True)
    assert torch.equal(dx_a, dx_b)
    for a, b in zip(gr_a, gr_b):
        assert torch.equal(a, b)
