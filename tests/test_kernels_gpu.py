"""GPU parity of each HIP kernel family against a plain torch fp32 reference of the same op
(computed on the host CPU).  fp32 mode is the exact-fp32 MFMA path (tolerance 1e-5
relative L2); bf16 mode is checked at bf16 tolerance (2e-2)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import _lib as L  # noqa: E402
from facevae_amd import ops  # noqa: E402

CL = torch.channels_last
TOL = {torch.float32: 1e-5, torch.bfloat16: 2e-2}


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def gen(seed):
    return torch.Generator().manual_seed(seed)


def conv_setup(x, w, k, dtype, ups=False, pro=False, slope=0.0, sigmoid=False, need_wt=False):
    N, C, Hi, Wi = x.shape
    cout = w.shape[0]
    H, W = (2 * Hi, 2 * Wi) if ups else (Hi, Wi)
    xb, cp = ops.to_nhwc(x.cuda(), dtype)
    d = ops.desc(dtype, N, H, W, cp, C, cout, cout, k, ups, pro, slope, sigmoid, 0)
    wk = torch.empty(L.query("fv_conv_wk_elems", ctypes.byref(d)), dtype=dtype, device="cuda")
    wt = torch.empty(L.query("fv_conv_wt_elems", ctypes.byref(d)), dtype=dtype, device="cuda") if need_wt else None
    wc = w.cuda().float().contiguous()
    L.call("fv_conv_weight_prep", ctypes.byref(d), wc.data_ptr(), None, wk.data_ptr(), L.ptr(wt), L.stream())
    return d, xb, wk, wt, (N, cout, H, W)


CONV_CASES = [
    # k, cin, cout, H, W, ups, pro
    (3, 32, 64, 12, 10, False, False),
    (3, 64, 128, 16, 16, False, True),
    (1, 256, 512, 8, 8, False, False),
    (7, 3, 64, 16, 16, False, False),
    (7, 64, 3, 16, 16, False, False),
    (3, 128, 64, 8, 8, True, False),
    (3, 32, 32, 8, 6, True, True),
    (3, 16, 32, 7, 9, False, False),
    # DMA-fed v2 path (bf16, cin % 64 == 0): big tiles, partial tiles, upsample, 1x1, 7x7
    (3, 256, 256, 16, 16, False, False),
    (3, 64, 128, 12, 20, False, False),
    (3, 128, 64, 10, 6, True, False),
    (7, 64, 3, 9, 13, False, False),
    (1, 512, 256, 6, 10, False, False),
    # 17..32 output rows on the v2 path (64-row co tile over a weight image of 32 rows before
    # wrows): a 1x1 128 -> 32 forward, the data gradient of 32 -> 128, a 3x3 with 24 outputs
    (1, 128, 32, 8, 64, False, False),
    (1, 32, 128, 16, 64, False, False),
    (3, 64, 24, 8, 16, False, False),
    # 7x7 halo path (bf16, W % 64 == 0): in_conv shape, out_conv shape (+ its dgrad)
    (7, 3, 64, 16, 64, False, False),
    (7, 64, 3, 8, 128, False, False),
    (7, 64, 3, 20, 64, False, False),   # out_conv wgrad: 3 ragged row segments
    (7, 64, 3, 64, 128, False, False),  # out_conv forward: a 64-row band per block (ring wraps 4x), below
    # halo-staged 3x3 (bf16, W % 64 == 0, H % 4 == 0): co tiles of 128 / 256 / 64, 2 column tiles
    (3, 64, 128, 8, 64, False, False),
    (3, 256, 256, 4, 64, False, False),
    (3, 128, 64, 12, 128, False, False),
    (3, 128, 64, 16, 64, False, False),    # 64-co tile on 8-row tiles (conv3_halo_fwd3<1, 8, ...>)
    # sub-pixel phases of upsample + 3x3 (bf16, power-of-two low-res side >= 16): UpBlock2D shapes
    (3, 128, 64, 16, 16, True, False),
    (3, 256, 128, 16, 32, True, False),
    # ... with low-res width 64: the sub-pixel weight gradient too
    (3, 128, 64, 8, 64, True, False),
    (3, 256, 128, 4, 64, True, False),
    # the 128-channel-input forward on the sliding band (conv3up_band_fwd): 2 co groups, 2 bands
    (3, 128, 128, 32, 64, True, False),
    # the full-size UpBlock2D convs (Generator.up at 256x256): fp32 parity of the large-P paths
    (3, 128, 64, 128, 128, True, False),
    (3, 256, 128, 64, 64, True, False),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd(case, dtype, monkeypatch):
    k, cin, cout, H, W, ups, pro = case
    if (k, cin, cout, H) == (7, 64, 3, 64):
        monkeypatch.setenv("FV_C7_BAND", "64")     # conv7_n3_fwd2: 16 row groups per block
    g = gen(100 + k + cin)
    x = torch.randn(2, cin, H, W, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g)
    sc = torch.rand(cin, generator=g) + 0.5
    sh = torch.randn(cin, generator=g) * 0.1
    slope = 0.2 if pro else 0.0
    xi = x
    if pro:
        xi = F.leaky_relu(x * sc[None, :, None, None] + sh[None, :, None, None], slope)
    if ups:
        xi = F.interpolate(xi, scale_factor=2, mode="nearest")
    ref = F.conv2d(xi, w, b, padding=k // 2)
    d, xb, wk, _, shp = conv_setup(x, w, k, dtype, ups, pro, slope)
    if cout % 4:
        d.out_nchw_f32 = 1
        y = torch.empty(shp, dtype=torch.float32, device="cuda")
    else:
        y = torch.empty(shp, dtype=dtype, device="cuda", memory_format=CL)
    scd, shd = sc.cuda(), sh.cuda()
    nb = L.query("fv_conv2d_stats_blocks", ctypes.byref(d))
    # records + a guard region: no launch writes a record past the nb the query sized (a partial
    # pixel tile's empty wave rows once did, an illegal address when the buffer ended a mapping)
    guard = 4 * 2 * cout
    pbuf = torch.full((nb * 2 * cout + guard,), 1234.5, device="cuda")
    part = pbuf[:nb * 2 * cout]
    L.call("fv_conv2d_fwd", ctypes.byref(d), xb.data_ptr(), wk.data_ptr(), b.cuda().data_ptr(),
           L.ptr(scd if pro else None), L.ptr(shd if pro else None), None, y.data_ptr(), part.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert bool((pbuf[nb * 2 * cout:] == 1234.5).all()), "BN records written past fv_conv2d_stats_blocks"
    assert rel(y.float(), ref) < TOL[dtype] * (1 if dtype == torch.float32 else 1.5)
    # block partials -> exact batch statistics
    if cout % 8 == 0:
        stats = torch.empty(3 * cout, dtype=torch.float64, device="cuda")
        ws = torch.empty(L.query("fv_bn_ws_bytes", cout) // 8, dtype=torch.float64, device="cuda")
        P = shp[0] * shp[2] * shp[3]
        L.call("fv_bn_stats_from_partials", part.data_ptr(), nb, L.query("fv_conv2d_stats_block_pixels",
               ctypes.byref(d)), P, cout, stats.data_ptr(), ws.data_ptr(), L.stream())
        s = stats.cpu().view(3, cout)
        # statistics come from the fp32 accumulators (before the bf16 rounding of y)
        yr = ref.permute(1, 0, 2, 3).reshape(cout, -1).double()
        assert torch.allclose(s[0], torch.full((cout,), float(P), dtype=torch.float64))
        t = 1e-5 if dtype == torch.float32 else 1e-2
        assert ((s[1] - yr.sum(1)).abs() / yr.abs().sum(1)).max() < t
        assert rel(s[2], (yr * yr).sum(1)) < t


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_bwd(case, dtype):
    k, cin, cout, H, W, ups, pro = case
    g = gen(200 + k + cin)
    x = torch.randn(2, cin, H, W, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    sc = torch.rand(cin, generator=g) + 0.5
    sh = torch.randn(cin, generator=g) * 0.1
    slope = 0.0
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = torch.zeros(cout, requires_grad=True)
    xi = xr
    if pro:
        xi = F.relu(xr * sc[None, :, None, None] + sh[None, :, None, None])
    if ups:
        xi = F.interpolate(xi, scale_factor=2, mode="nearest")
    out = F.conv2d(xi, wr, br, padding=k // 2)
    gy = torch.randn(out.shape, generator=g)
    (out * gy).sum().backward()
    d, xb, wk, wt, shp = conv_setup(x, w, k, dtype, ups, pro, slope, need_wt=True)
    ldd = ops.pad_pow2(cout)
    gyb = torch.zeros((2, ldd, shp[2], shp[3]), dtype=dtype, device="cuda").contiguous(memory_format=CL)
    gyb[:, :cout] = gy.cuda().to(dtype)
    # weight + bias gradient
    slab = torch.empty(L.query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), device="cuda")
    bslab = torch.empty(L.query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), device="cuda")
    scd, shd = sc.cuda(), sh.cuda()
    L.call("fv_conv2d_bwd_weight", ctypes.byref(d), xb.data_ptr(), L.ptr(scd if pro else None),
           L.ptr(shd if pro else None), gyb.data_ptr(), ldd, slab.data_ptr(), bslab.data_ptr(), L.stream())
    dw = torch.empty(cout, cin, k, k, device="cuda")
    db = torch.empty(cout, device="cuda")
    L.call("fv_conv2d_wgrad_reduce", ctypes.byref(d), slab.data_ptr(), bslab.data_ptr(), dw.data_ptr(),
           db.data_ptr(), L.stream())
    torch.cuda.synchronize()
    tol = TOL[dtype] * (1 if dtype == torch.float32 else 1.5)
    assert rel(dw, wr.grad) < tol
    assert rel(db, br.grad) < tol
    # data gradient (w.r.t. the conv input, before the prologue)
    if not pro and ups and L.query("fv_conv2d_dgrad_lowres", ctypes.byref(d)):
        dx = torch.empty((2, xb.shape[1], H, W), dtype=dtype, device="cuda", memory_format=CL)
        L.call("fv_conv2d_bwd_data", ctypes.byref(d), gyb.data_ptr(), ldd, wt.data_ptr(), dx.data_ptr(), L.stream())
        torch.cuda.synchronize()
        assert rel(dx[:, :cin].float(), xr.grad) < tol
    elif not pro:
        dx = torch.empty((2, xb.shape[1], shp[2], shp[3]), dtype=dtype, device="cuda", memory_format=CL)
        L.call("fv_conv2d_bwd_data", ctypes.byref(d), gyb.data_ptr(), ldd, wt.data_ptr(), dx.data_ptr(), L.stream())
        if ups:
            src = torch.empty((2, xb.shape[1], H, W), dtype=dtype, device="cuda", memory_format=CL)
            L.call("fv_upsample2x_bwd", L.dtype_code(dtype), dx.data_ptr(), 2, H, W, xb.shape[1], src.data_ptr(),
                   L.stream())
            dx = src
        torch.cuda.synchronize()
        assert rel(dx[:, :cin].float(), xr.grad) < tol


def test_spectral_norm():
    g = gen(7)
    w = torch.randn(64, 32, 3, 3, generator=g)
    u = F.normalize(torch.randn(64, generator=g), dim=0)
    v = F.normalize(torch.randn(288, generator=g), dim=0)
    wm = w.reshape(64, -1)
    v2 = F.normalize(wm.t() @ u, dim=0)
    u2 = F.normalize(wm @ v2, dim=0)
    sig = torch.dot(u2, wm @ v2)
    wc, uc, vc = w.cuda(), u.cuda(), v.cuda()
    sigma = ops.spectral_norm_fwd(wc, uc, vc, True)
    torch.cuda.synchronize()
    assert rel(uc, u2) < 1e-5 and rel(vc, v2) < 1e-5
    assert abs(sigma.item() - sig.item()) < 1e-5 * sig.item()
    # backward through W / sigma (u, v constants)
    wr = w.clone().requires_grad_(True)
    gsn = torch.randn(64, 32, 3, 3, generator=g)
    (wr / torch.dot(u2, wr.reshape(64, -1) @ v2) * gsn).sum().backward()
    gc = gsn.cuda().contiguous()
    ops.spectral_norm_bwd(wc, gc, uc, vc, sigma)
    torch.cuda.synchronize()
    assert rel(gc, wr.grad) < 1e-5


@pytest.mark.parametrize("uses", ["kl", "z", "kl+mu", "kl_twice"])
@pytest.mark.parametrize("H", [8, 6])
def test_reparam_kl_gradient_routes(H, uses):
    """The KL gradient folded into the reparameterisation backward (fv_reparam_kl_bwd): KL
    alone, z alone, KL plus another loss on mu (dmu and the folded term together), KL counted
    twice -- each against torch autograd on the same fp32 values."""
    g = gen(12)
    N, Lc = 2, 16
    h = torch.randn(N, 2 * Lc, H, H, generator=g) * 0.5
    eps = torch.randn(N, Lc, H, H, generator=g)
    gz = torch.randn(N, Lc, H, H, generator=g)

    def loss(mu, ls, z, kl):
        if uses == "kl":
            return 2.0 * kl(mu, ls)
        if uses == "z":
            return (z.float() * gz.to(z.device)).sum()
        if uses == "kl+mu":
            return kl(mu, ls) + (mu.float() * gz.to(mu.device)).sum()
        return kl(mu, ls) + 0.5 * kl(mu, ls)

    hr = h.clone().requires_grad_(True)
    mu_r, ls_r = hr[:, :Lc], hr[:, Lc:]
    loss(mu_r, ls_r, mu_r + torch.exp(ls_r) * eps,
         lambda m, s: torch.mean(-0.5 - s + 0.5 * m ** 2 + 0.5 * torch.exp(2 * s))).backward()
    hc = h.cuda().contiguous(memory_format=CL).requires_grad_(True)
    mu, ls, z = ops.reparameterise(hc, eps.cuda(), torch.float32)
    loss(mu, ls, z, lambda m, s: fv.KLDivergenceLoss()((m, s))).backward()
    torch.cuda.synchronize()
    assert rel(hc.grad, hr.grad) < 1e-5


@pytest.mark.parametrize("H", [8, 6])          # 8: tiled reparam + fused KL; 6: hw % 32 != 0 fallback
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_losses_and_reparam(dtype, H):
    g = gen(11)
    N, Lc = 2, 16
    h = torch.randn(N, 2 * Lc, H, H, generator=g) * 0.5
    eps = torch.randn(N, Lc, H, H, generator=g)
    hr = h.to(dtype).float().clone().requires_grad_(True)
    mu_r, ls_r = hr[:, :Lc], hr[:, Lc:]
    z_r = mu_r + torch.exp(ls_r) * eps
    K_r = torch.mean(-0.5 - ls_r + 0.5 * mu_r ** 2 + 0.5 * torch.exp(2 * ls_r), dim=-1).mean()
    gz = torch.randn(z_r.shape, generator=g)
    ((z_r * gz).sum() + 3.0 * K_r).backward()
    hc = h.detach().cuda().to(dtype).contiguous(memory_format=CL).requires_grad_(True)
    mu, ls, z = ops.reparameterise(hc, eps.cuda(), dtype)
    K = fv.KLDivergenceLoss()((mu, ls))
    ((z.float() * gz.cuda()).sum() + 3.0 * K).backward()
    torch.cuda.synchronize()
    tol = TOL[dtype]
    assert rel(z.float(), z_r) < tol
    assert abs(K.item() - K_r.item()) < tol * abs(K_r.item())
    # the KL reduced inside the reparameterisation pass == the standalone KL kernel
    K2 = fv.KLDivergenceLoss()((mu.detach().clone(), ls.detach().clone()))
    assert abs(K.item() - K2.item()) < 1e-5 * abs(K2.item())
    assert rel(hc.grad.float(), hr.grad) < tol * 2
    assert torch.equal(mu.float().cpu(), h.to(dtype).float()[:, :Lc]) and torch.equal(
        ls.float().cpu(), h.to(dtype).float()[:, Lc:])
    # MSE / L1 on fp32 NCHW images
    a = torch.rand(2, 3, 16, 16, generator=g)
    b = torch.rand(2, 3, 16, 16, generator=g)
    for fn_ours, fn_ref in ((fv.ReconLoss(), lambda p: F.mse_loss(p[0], p[1])),):
        ar, br_ = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
        lr_ = fn_ref((ar, br_))
        lr_.backward()
        ac, bc = a.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
        lo = fn_ours((ac, bc))
        lo.backward()
        assert abs(lo.item() - lr_.item()) < 1e-6 * lr_.item()
        assert rel(ac.grad, ar.grad) < 1e-6 and rel(bc.grad, br_.grad) < 1e-6
    ar, br_ = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
    F.l1_loss(ar, br_).backward()
    ac, bc = a.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    lo = fv.L1Loss()(ac, bc)
    lo.backward()
    assert abs(lo.item() - F.l1_loss(a, b).item()) < 1e-6
    assert rel(ac.grad, ar.grad) < 1e-6


def test_adam_matches_torch():
    g = gen(5)
    ps = [torch.randn(s, generator=g) for s in (10, 5000, 4096 * 3 + 7)]
    gs = [[torch.randn(p.shape, generator=g) for p in ps] for _ in range(3)]
    ref = [p.clone().requires_grad_(True) for p in ps]
    ours = [p.cuda().requires_grad_(True) for p in ps]
    o_ref = torch.optim.Adam(ref, lr=5e-3, betas=(0.5, 0.999))
    o_ours = fv.Adam(ours, lr=5e-3, betas=(0.5, 0.999))
    for step in range(3):
        for p, gg in zip(ref, gs[step]):
            p.grad = gg.clone()
        for p, gg in zip(ours, gs[step]):
            p.grad = gg.cuda()
        o_ref.step()
        o_ours.step()
    torch.cuda.synchronize()
    for a, b in zip(ours, ref):
        assert rel(a.detach(), b.detach()) < 1e-6
    sa, sb = o_ours.state_dict(), o_ref.state_dict()
    assert sa["state"][1]["step"].item() == sb["state"][1]["step"].item() == 3
    assert rel(sa["state"][2]["exp_avg_sq"], sb["state"][2]["exp_avg_sq"]) < 1e-6


def test_error_is_reported_not_aborted():
    d = ops.desc(torch.float32, 1, 8, 8, 12, 12, 16, 16, 3)    # cin 12 is not a power of two
    with pytest.raises(L.FaceVAELibError, match="power of two"):
        L.call("fv_conv2d_fwd", ctypes.byref(d), 1, 1, None, None, None, None, 1, None, L.stream())


@pytest.mark.parametrize("case", ["demod", "plain_untied", "demod_128to64"])
def test_conv_transpose_elr(case):
    """ConvTranspose2dELR k4 s2 p1 (models_utils.py:404-516) on the sub-pixel kernels vs the
    oracle restatement (oracle.convt_elr, pinned to the reference by
    tests/golden/convt_elr.pt) in fp32 on the CPU: output, input / weight / bias gradients at
    bf16 tolerance.  No activation module here: a ReLU / LeakyReLU (a torch module applied
    after the kernel, as in the reference) flips its mask on ~0.2 % of near-zero outputs
    between a bf16 and an fp32 forward, which alone moves the gradients by ~3 %."""
    from oracle import facevae_cpu as O      # checker only
    inch, outch, norm, ub, slope, hw = {
        "demod": (64, 64, "demod", None, None, (64, 64)),
        "plain_untied": (64, 128, None, (128, 128), None, (64, 64)),
        "demod_128to64": (128, 64, "demod", None, None, (32, 128)),
    }[case]
    act = None if slope is None else (torch.nn.ReLU() if slope == 0.0 else torch.nn.LeakyReLU(slope))
    torch.manual_seed(0)
    m = fv.ConvTranspose2dELR(inch, outch, 4, 2, 1, norm=norm, ub=ub, act=act)
    with torch.no_grad():
        m.bias.normal_(generator=gen(5))
    if case == "demod":
        gold = torch.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                                     "convt_elr.pt"), weights_only=True)["gpu_init"]
        assert abs(m.weight.double().sum().item() - gold["sum"].item()) < 1e-9   # reference init
    w0, b0 = m.weight.detach().clone(), m.bias.detach().clone()
    x = torch.randn(2, inch, *hw, generator=gen(6))
    g = torch.randn(2, outch, 2 * hw[0], 2 * hw[1], generator=gen(7))
    m = m.cuda()
    xc = x.cuda().requires_grad_(True)
    y = m(xc)
    y.float().backward(g.cuda())
    torch.cuda.synchronize()
    wr, br, xr = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True), x.clone().requires_grad_(True)
    yr = O.convt_elr(xr, wr, br, 2, 1, norm, m.weightgain, slope)
    yr.backward(g)
    dev = {"y": rel(y.float(), yr.detach()), "dx": rel(xc.grad, xr.grad), "dw": rel(m.weight.grad, wr.grad),
           "db": rel(m.bias.grad, br.grad)}
    print(f"\n[convT {case}] rel-L2 vs oracle: {dev}")
    assert max(dev.values()) < TOL[torch.bfloat16], dev


CONVT_FIXTURES = {
    "demod_leaky": (6, 8, 4, 2, 1, "demod", None, 0.2),
    "plain_untied": (4, 8, 4, 2, 1, None, (10, 12), None),
    "demod_relu_k3s1": (5, 8, 3, 1, 1, "demod", None, 0.0),
}


@pytest.mark.parametrize("name", list(CONVT_FIXTURES))
def test_conv_transpose_elr_fp32_matches_reference(name):
    """Every reference fixture case of ConvTranspose2dELR (odd sizes, k3 s1, untied bias) in fp32
    parity mode on the direct kernels of convt.hip: 1e-4 relative (north_star 1e-3)."""
    g = torch.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "convt_elr.pt"),
                   weights_only=True)[name]
    inch, outch, k, s, p, norm, ub, slope = CONVT_FIXTURES[name]
    act = None if slope is None else (torch.nn.ReLU() if slope == 0.0 else torch.nn.LeakyReLU(slope))
    m = fv.ConvTranspose2dELR(inch, outch, k, s, p, norm=norm, ub=ub, act=act)
    with torch.no_grad():
        m.weight.copy_(g["weight"])
        m.bias.copy_(g["bias"])
    m = m.cuda().set_compute_dtype(torch.float32)
    x = g["x"].cuda().requires_grad_(True)
    y = m(x)
    y.float().backward(g["g"].cuda())
    torch.cuda.synchronize()
    assert rel(y.float(), g["y"]) < 1e-4
    assert rel(x.grad, g["dx"]) < 1e-4
    assert rel(m.weight.grad, g["dweight"]) < 1e-4
    assert rel(m.bias.grad, g["dbias"]) < 1e-4


@pytest.mark.parametrize("name,mode", [("mod_demod_leaky", torch.float32), ("mod_plain_k3s1", torch.float32),
                                       ("mod_demod_leaky", torch.bfloat16)])
def test_conv_transpose_elr_modulated_matches_reference(name, mode):
    """Per-sample affine modulation (wsize > 0, forward(x, w)): modulation and demodulation as
    channel scales around the shared-weight kernel vs the reference's grouped conv."""
    g = torch.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "convt_elr.pt"),
                   weights_only=True)[name]
    inch, outch, k, s, p, norm, wsize, slope = {"mod_demod_leaky": (6, 8, 4, 2, 1, "demod", 5, 0.2),
                                                "mod_plain_k3s1": (5, 8, 3, 1, 1, None, 4, None)}[name]
    act = None if slope is None else torch.nn.LeakyReLU(slope)
    m = fv.ConvTranspose2dELR(inch, outch, k, s, p, wsize=wsize, norm=norm, act=act)
    m.load_state_dict(g["init"])
    m = m.cuda().set_compute_dtype(mode)
    x, w = g["x"].cuda().requires_grad_(True), g["w"].cuda().requires_grad_(True)
    y = m(x, w)
    y.float().backward(g["g"].cuda())
    torch.cuda.synchronize()
    tol = 1e-4 if mode == torch.float32 else 3e-2
    assert rel(y.float(), g["y"]) < tol
    assert rel(x.grad, g["dx"]) < tol and rel(w.grad, g["dw"]) < tol
    for kk, prm in m.named_parameters():
        assert rel(prm.grad, g["grads"][kk]) < tol * 3, kk


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 64, 16, 32), (3, 128, 8, 8)])
def test_bn_act_bwd_pooled(shape, dtype):
    """DownBlock2D's BN backward (BN -> ReLU -> AvgPool2d(2)): the 2x2-quad reduce + apply
    kernels against torch autograd of batch_norm(training) -> relu -> avg_pool2d on the same
    (rounded) operands; dgamma, dbeta and dx."""
    N, C, H, W = shape
    g = gen(7 + C)
    y = torch.randn(N, C, H, W, generator=g) * 2 + 0.3
    gam = torch.rand(C, generator=g) + 0.5
    bet = torch.randn(C, generator=g) * 0.2
    dout = torch.randn(N, C, H // 2, W // 2, generator=g)
    y = y.to(dtype).float()
    dout = dout.to(dtype).float()
    yr = y.double().requires_grad_(True)
    gr, br = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    z = F.avg_pool2d(F.relu(F.batch_norm(yr, None, None, gr, br, training=True, eps=1e-5)), 2)
    z.backward(dout.double())
    mean = y.double().mean(dim=(0, 2, 3))
    var = y.double().var(dim=(0, 2, 3), unbiased=False)
    inv = (var + 1e-5).rsqrt()
    yd = y.to(dtype).cuda().contiguous(memory_format=CL)
    dd = dout.to(dtype).cuda().contiguous(memory_format=CL)
    dev = lambda t: t.float().cuda().contiguous()
    dg = torch.empty(C, device="cuda")
    db = torch.empty(C, device="cuda")
    k = torch.empty(2 * C, device="cuda")
    ws = torch.empty(L.query("fv_bn_ws_bytes", C) // 8, dtype=torch.float64, device="cuda")
    m_, i_, g_, b_ = dev(mean), dev(inv), dev(gam), dev(bet)
    L.call("fv_bn_act_bwd_reduce_finalize", L.dtype_code(dtype), dd.data_ptr(), yd.data_ptr(), N, H, W, C, C,
           m_.data_ptr(), i_.data_ptr(), g_.data_ptr(), b_.data_ptr(), 0.0, 1, N * H * W, dg.data_ptr(),
           db.data_ptr(), k.data_ptr(), ws.data_ptr(), L.stream())
    dx = torch.empty((N, C, H, W), dtype=dtype, device="cuda", memory_format=CL)
    L.call("fv_bn_act_bwd_apply", L.dtype_code(dtype), dd.data_ptr(), yd.data_ptr(), N, H, W, C, C,
           m_.data_ptr(), i_.data_ptr(), g_.data_ptr(), b_.data_ptr(), 0.0, 1, k.data_ptr(), None, dx.data_ptr(),
           L.stream())
    torch.cuda.synchronize()
    tol = 1e-4 if dtype == torch.float32 else 1e-2
    assert rel(dg, gr.grad) < tol and rel(db, br.grad) < tol
    assert rel(dx.float(), yr.grad) < tol * 2
    # the comm-path reduce (sums only, all-reduced elsewhere) gives the same sums
    red = torch.empty(2 * C, dtype=torch.float64, device="cuda")
    L.call("fv_bn_act_bwd_reduce", L.dtype_code(dtype), dd.data_ptr(), yd.data_ptr(), N, H, W, C, C, m_.data_ptr(),
           i_.data_ptr(), g_.data_ptr(), b_.data_ptr(), 0.0, 1, red.data_ptr(), ws.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert rel(red[:C], br.grad) < tol and rel(red[C:], gr.grad) < tol


@pytest.mark.parametrize("res", [False, True])
def test_conv3x3_64ch_with_residual(res):
    """a 64 -> 64 3x3 conv (a 64-channel ResBlock2D conv) has the shape of the 64-channel
    band kernel (conv3c64_fwd), which has no residual epilogue; with a residual the launch must run
    the generic DMA-fed kernel on the same prepared weights instead of failing."""
    N, C, H, W = 2, 64, 64, 64
    g = gen(77)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(C, C, 3, 3, generator=g) / (C * 9) ** 0.5
    b = torch.randn(C, generator=g)
    r = torch.randn(N, C, H, W, generator=g)
    dtype = torch.bfloat16
    d, xb, wk, _, shp = conv_setup(x, w, 3, dtype)
    rb = r.cuda().to(dtype).contiguous(memory_format=CL)
    y = torch.empty(shp, dtype=dtype, device="cuda", memory_format=CL)
    L.call("fv_conv2d_fwd", ctypes.byref(d), xb.data_ptr(), wk.data_ptr(), b.cuda().data_ptr(), None, None,
           L.ptr(rb if res else None), y.data_ptr(), None, L.stream())
    torch.cuda.synchronize()
    xq = xb.float().cpu()
    ref = F.conv2d(xq, w, b, padding=1) + (rb.float().cpu() if res else 0)
    assert rel(y.float(), ref) < 1e-2


@pytest.mark.parametrize("spb", [1, 4])
def test_up_wgrad_splits(spb, monkeypatch):
    """UpBlock2D weight gradient (conv3_up_wgrad: sub-pixel phases on the sliding-row structure)
    at 3 images x 2 output strips = 6 units, 1 or 4 units per block (the last split ragged), vs
    torch fp32 (the CONV_CASES cover it at N = 2 and the full UpBlock2D sizes)."""
    monkeypatch.setenv("FV_UPW_SPB", str(spb))
    N, cin, cout, Hi, Wi = 3, 128, 64, 8, 64
    g = gen(777)
    x = torch.randn(N, cin, Hi, Wi, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    wr = w.clone().requires_grad_(True)
    br = torch.zeros(cout, requires_grad=True)
    out = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), wr, br, padding=1)
    gy = torch.randn(out.shape, generator=g)
    (out * gy).sum().backward()
    d, xb, wk, wt, shp = conv_setup(x, w, 3, torch.bfloat16, True, need_wt=True)
    gyb = gy.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    slab = torch.empty(L.query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)), device="cuda")
    bslab = torch.empty(L.query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), device="cuda")
    L.call("fv_conv2d_bwd_weight", ctypes.byref(d), xb.data_ptr(), None, None, gyb.data_ptr(), cout,
           slab.data_ptr(), bslab.data_ptr(), L.stream())
    dw = torch.empty(cout, cin, 3, 3, device="cuda")
    db = torch.empty(cout, device="cuda")
    L.call("fv_conv2d_wgrad_reduce", ctypes.byref(d), slab.data_ptr(), bslab.data_ptr(), dw.data_ptr(),
           db.data_ptr(), L.stream())
    torch.cuda.synchronize()
    assert L.query("fv_conv2d_wgrad_nsplit", ctypes.byref(d)) == (6 + spb - 1) // spb
    assert rel(dw, wr.grad) < TOL[torch.bfloat16] * 1.5
    assert rel(db, br.grad) < TOL[torch.bfloat16] * 1.5


# 1x1 convs on the pixel-stream kernel (conv.hip conv1x1_stream): the mid convs' forward and
# data-gradient shapes -- one tile per stream, several tiles per stream (the t + 2 DMA under the
# stores), 2 co groups -- bit-identical to conv_fwd_v2's 256 x 256 tile (same k order, same
# epilogue: FV_C1S=0) and within bf16 tolerance of the torch fp32 conv
C1S_CASES = [
    # cin, cout, N, H, W
    (256, 512, 2, 16, 64),      # 16 pixel tiles, 2 co groups
    (256, 256, 16, 64, 64),     # 512 tiles: 2 per stream
    (512, 256, 8, 64, 64),      # K = 512 (AFE.mid_conv's data gradient shape): 64-pixel tiles
    (256, 512, 24, 64, 64),     # 768 tiles, 2 co groups: 6 per stream
]


@pytest.mark.parametrize("bp", ["64", "128"])
@pytest.mark.parametrize("case", C1S_CASES)
def test_conv1x1_stream(case, bp, monkeypatch):
    cin, cout, N, H, W = case
    monkeypatch.setenv("FV_C1S_BP", bp)         # 4 slots of 32 KB / 2 slots of 64 KB
    g = gen(300 + cin + N)
    x = torch.randn(N, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5
    b = torch.randn(cout, generator=g)
    d, xb, wk, wt, shp = conv_setup(x, w, 1, torch.bfloat16, need_wt=True)
    bc = b.cuda()
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("FV_C1S", mode)
        y = torch.empty(shp, dtype=torch.bfloat16, device="cuda", memory_format=CL)
        L.call("fv_conv2d_fwd", ctypes.byref(d), xb.data_ptr(), wk.data_ptr(), bc.data_ptr(), None, None, None,
               y.data_ptr(), None, L.stream())
        gy = torch.randn(shp, generator=gen(7)).cuda().to(torch.bfloat16).contiguous(memory_format=CL)
        dx = torch.empty((N, cin, H, W), dtype=torch.bfloat16, device="cuda", memory_format=CL)
        L.call("fv_conv2d_bwd_data", ctypes.byref(d), gy.data_ptr(), cout, wt.data_ptr(), dx.data_ptr(), L.stream())
        torch.cuda.synchronize()
        outs[mode] = (y, dx, gy)
    (y1, dx1, gy), (y0, dx0, _) = outs["1"], outs["0"]
    assert torch.equal(y1, y0) and torch.equal(dx1, dx0)
    xq = xb.float().cpu()
    wq = w.cuda().to(torch.bfloat16).float().cpu()
    ref = F.conv2d(xq, wq, b)
    assert rel(y1.float().cpu(), ref) < TOL[torch.bfloat16]
    dref = F.conv_transpose2d(gy.float().cpu(), wq)
    assert rel(dx1.float().cpu(), dref) < TOL[torch.bfloat16]


@pytest.mark.parametrize("shape", [(2, 16, 64), (4, 32, 128)])
def test_in_conv_wgrad_packed_layout(shape, monkeypatch):
    """AFE.in_conv's weight gradient (7x7, 3 -> 64) with k packed as (row, 4 taps x 4 channels)
    -- 14 m-tiles instead of 25 -- is bit-identical to the 8-channel padded layout (the same
    pixel sums per output element; FV_WG7_PACK=0) and matches torch fp32 at bf16 tolerance."""
    N, H, W = shape
    g = gen(41 + H)
    x = torch.rand(N, 3, H, W, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) / 147 ** 0.5
    gy = torch.randn(N, 64, H, W, generator=g)
    d, xb, wk, _, shp = conv_setup(x, w, 7, torch.bfloat16)
    gyb = gy.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    res = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("FV_WG7_PACK", mode)
        slab = torch.full((L.query("fv_conv2d_wgrad_slab_elems", ctypes.byref(d)),), float("nan"), device="cuda")
        bslab = torch.empty(L.query("fv_conv2d_wgrad_bias_slab_elems", ctypes.byref(d)), device="cuda")
        L.call("fv_conv2d_bwd_weight", ctypes.byref(d), xb.data_ptr(), None, None, gyb.data_ptr(), 64,
               slab.data_ptr(), bslab.data_ptr(), L.stream())
        dw = torch.empty(64, 3, 7, 7, device="cuda")
        db = torch.empty(64, device="cuda")
        L.call("fv_conv2d_wgrad_reduce", ctypes.byref(d), slab.data_ptr(), bslab.data_ptr(), dw.data_ptr(),
               db.data_ptr(), L.stream())
        torch.cuda.synchronize()
        res[mode] = (dw.cpu(), db.cpu())
    assert torch.equal(res["1"][0], res["0"][0]) and torch.equal(res["1"][1], res["0"][1])
    xq = xb[:, :3].float().cpu()
    wr = w.clone().requires_grad_(True)
    (F.conv2d(xq, wr, padding=3) * gyb.float().cpu()).sum().backward()
    assert rel(res["1"][0], wr.grad) < TOL[torch.bfloat16]
    assert torch.isfinite(res["1"][0]).all()
