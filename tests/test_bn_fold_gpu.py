"""BN record folds, bit-reproducibility and values.  The conv-record fold runs its second
level inside the first level's launch (bn.hip fold16_part_kernel: chunk rows stored sc1, an
arrival ticket per 16-channel group, the group's last arriver sums the chunk rows after one
agent acquire), so its result must not depend on arrival order or placement: every entry
point is checked against a float64 torch reference and for bit-identical results over
repeated launches, alone and with a matmul stream competing for the CUs.  The backward-reduce
and tensor-statistics folds (separate fold launch) are held to the same bar.  Shapes cover
pooled / unpooled backward, a partial 16-channel group (C = 8), few rows, and the
256-channel res layer (1024 rows)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
from facevae_amd import _lib as L  # noqa: E402

CL = torch.channels_last


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _repeat_under_load(fn, reps=6):
    """fn() -> tuple of device tensors; run reps times alone and reps times beside a
    matmul stream; every run bit-identical to the first."""
    first = [t.clone() for t in fn()]
    torch.cuda.synchronize()
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    for i in range(2 * reps):
        if i >= reps:
            with torch.cuda.stream(side):
                for _ in range(3):
                    a = (a @ a).clamp_(-1, 1)
        out = fn()
        torch.cuda.synchronize()
        for x, y in zip(out, first):
            assert torch.equal(x, y), f"run {i}: fold result changed"
    return first


@pytest.mark.parametrize("shape", [(32, 256, 64, 64), (2, 64, 16, 32), (1, 256, 2, 4), (2, 8, 8, 8)])
@pytest.mark.parametrize("pool", [0, 1])
def test_bwd_reduce_fold(shape, pool):
    N, C, H, W = shape
    g = torch.Generator().manual_seed(11 + C + pool)
    y = (torch.randn(N, C, H, W, generator=g) * 2 + 0.3).to(torch.bfloat16).float()
    gam = torch.rand(C, generator=g) + 0.5
    bet = torch.randn(C, generator=g) * 0.2
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    dout = torch.randn(N, C, Ho, Wo, generator=g).to(torch.bfloat16).float()
    yr = y.double().requires_grad_(True)
    gr, br = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    z = F.relu(F.batch_norm(yr, None, None, gr, br, training=True, eps=1e-5))
    if pool:
        z = F.avg_pool2d(z, 2)
    z.backward(dout.double())
    mean = y.double().mean(dim=(0, 2, 3))
    inv = (y.double().var(dim=(0, 2, 3), unbiased=False) + 1e-5).rsqrt()
    yd = y.to(torch.bfloat16).cuda().contiguous(memory_format=CL)
    dd = dout.to(torch.bfloat16).cuda().contiguous(memory_format=CL)
    dev = lambda t: t.float().cuda().contiguous()
    m_, i_, g_, b_ = dev(mean), dev(inv), dev(gam), dev(bet)
    ws = torch.empty(L.query("fv_bn_ws_bytes", C) // 8, dtype=torch.float64, device="cuda")
    bf = L.dtype_code(torch.bfloat16)

    def fin():
        dg, db, k = (torch.full((n,), float("nan"), device="cuda") for n in (C, C, 2 * C))
        L.call("fv_bn_act_bwd_reduce_finalize", bf, dd.data_ptr(), yd.data_ptr(), N, H, W, C, C, m_.data_ptr(),
               i_.data_ptr(), g_.data_ptr(), b_.data_ptr(), 0.0, pool, N * H * W, dg.data_ptr(), db.data_ptr(),
               k.data_ptr(), ws.data_ptr(), L.stream())
        return dg, db, k

    def sums():
        red = torch.full((2 * C,), float("nan"), dtype=torch.float64, device="cuda")
        L.call("fv_bn_act_bwd_reduce", bf, dd.data_ptr(), yd.data_ptr(), N, H, W, C, C, m_.data_ptr(),
               i_.data_ptr(), g_.data_ptr(), b_.data_ptr(), 0.0, pool, red.data_ptr(), ws.data_ptr(), L.stream())
        return (red,)

    dg, db, k = _repeat_under_load(fin)
    (red,) = _repeat_under_load(sums)
    tol = 2e-3
    assert rel(dg, gr.grad) < tol and rel(db, br.grad) < tol
    assert rel(red[:C], br.grad) < tol and rel(red[C:], gr.grad) < tol
    cnt = N * H * W
    assert rel(k[:C], br.grad / cnt) < tol and rel(k[C:], gr.grad / cnt) < tol


@pytest.mark.parametrize("nrec,C", [(1024, 256), (4096, 128), (300, 64), (257, 512)])
def test_record_fold_in_launch(nrec, C):
    """conv-epilogue records [nrec][2][C] fp32 (sum, sum of squares of `bp` pixels each) ->
    stats / finalize in one launch (level 1 chunk partials + level 2 by the last arrivers)."""
    g = torch.Generator().manual_seed(nrec + C)
    bp = 128
    x = torch.randn(nrec, bp, C, generator=g) * 1.5 + 0.2
    rec = torch.stack([x.sum(1), (x * x).sum(1)], dim=1).float()       # [nrec][2][C]
    P = nrec * bp
    S, Q = rec[:, 0].double().sum(0), rec[:, 1].double().sum(0)
    mean = S / P
    var = Q / P - mean * mean
    gam = torch.rand(C, generator=g) + 0.5
    bet = torch.randn(C, generator=g) * 0.2
    rd = rec.cuda().contiguous()
    ws = torch.empty(L.query("fv_bn_ws_bytes", C) // 8, dtype=torch.float64, device="cuda")
    gd, bd = gam.cuda(), bet.cuda()

    def stats():
        st = torch.full((3 * C,), float("nan"), dtype=torch.float64, device="cuda")
        L.call("fv_bn_stats_from_partials", rd.data_ptr(), nrec, bp, P, C, st.data_ptr(), ws.data_ptr(), L.stream())
        return (st,)

    def fin():
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbt = torch.zeros(1, dtype=torch.int64, device="cuda")
        sm, si, sc, sh = (torch.full((C,), float("nan"), device="cuda") for _ in range(4))
        L.call("fv_bn_stats_finalize_partials", rd.data_ptr(), nrec, bp, P, C, gd.data_ptr(), bd.data_ptr(), 1e-5,
               0.1, rm.data_ptr(), rv.data_ptr(), nbt.data_ptr(), sm.data_ptr(), si.data_ptr(), sc.data_ptr(),
               sh.data_ptr(), ws.data_ptr(), L.stream())
        return rm, rv, nbt, sm, si, sc, sh

    (st,) = _repeat_under_load(stats)
    rm, rv, nbt, sm, si, sc, sh = _repeat_under_load(fin)
    assert torch.all(st[:C].cpu() == P)
    assert rel(st[C:2 * C], S) < 1e-12 and rel(st[2 * C:], Q) < 1e-12
    inv = (var + 1e-5).rsqrt()
    assert rel(sm, mean) < 1e-6 and rel(si, inv) < 1e-6
    assert rel(sc, gam.double() * inv) < 1e-6 and rel(sh, bet.double() - mean * gam.double() * inv) < 1e-5
    assert rel(rm, 0.1 * mean) < 1e-6 and rel(rv, 0.9 + 0.1 * var * P / (P - 1)) < 1e-6
    assert int(nbt.item()) == 1


@pytest.mark.parametrize("P,C", [(8192, 256), (100, 64), (3, 16)])
def test_tensor_stats_fold(P, C):
    g = torch.Generator().manual_seed(P + C)
    x = (torch.randn(P, C, generator=g) * 1.3 - 0.4).to(torch.bfloat16)
    xd = x.cuda().contiguous()
    xf = x.double()
    ws = torch.empty(L.query("fv_bn_ws_bytes", C) // 8, dtype=torch.float64, device="cuda")

    def stats():
        st = torch.full((3 * C,), float("nan"), dtype=torch.float64, device="cuda")
        L.call("fv_bn_stats_tensor", L.dtype_code(torch.bfloat16), xd.data_ptr(), P, C, C, st.data_ptr(),
               ws.data_ptr(), L.stream())
        return (st,)

    (st,) = _repeat_under_load(stats)
    assert torch.all(st[:C].cpu() == P)
    assert rel(st[C:2 * C], xf.sum(0)) < 1e-6 and rel(st[2 * C:], (xf * xf).sum(0)) < 1e-6
