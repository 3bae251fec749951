"""GPU parity of the AFE 3-D trunk: the conv3d kernels against torch fp32
references on the same (bf16-rounded) operands, ResBlock3D / AFE against the reference
fixtures (tests/golden/afe3d.pt) and, at the real trunk shape, against the CPU oracle.

Tolerances: fp32 parity mode (direct kernels, fp32 FMA) 1e-5 per kernel, 1e-4 per block (the
north_star 1e-3 bar with margin).  bf16 kernels: fp32 accumulation of bf16 operands, output
rounded to bf16 -> rel-L2 <= 4e-3 and elementwise |d| <= 1.6e-2 * max|ref| (one bf16 ulp is
2^-8 relative); blocks in bf16 are reported and gated loosely (bf16 rounding of every
activation, as the 2-D path)."""
import ctypes
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import _lib as L, ops3d  # noqa: E402
from oracle import facevae_cpu as O  # noqa: E402  (checker only)

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CL3 = torch.channels_last_3d


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def maxd(a, b):
    return (a.detach().double().cpu() - b.detach().double().cpu()).abs().max().item()


def rnd(t, dtype):
    return t.to(dtype).float()


class _W:
    def __init__(self, w):
        self.weight = w


def run_conv3d(x, w, b, res=None, dtype=torch.bfloat16, stats=False):
    N, C, D, H, W = x.shape
    d = ops3d.desc3(dtype, N, D, H, W, C, w.shape[0])
    cs = ops3d.Conv3dState(_W(w.cuda().contiguous()), d, "cuda", True)
    xb = x.cuda().to(dtype).contiguous(memory_format=CL3)
    rb = res.cuda().to(dtype).contiguous(memory_format=CL3) if res is not None else None
    y, rec = ops3d.conv3d_forward(cs, xb, b.cuda() if b is not None else None, res=rb, stats=stats)
    return cs, xb, y, rec


@pytest.mark.parametrize("shape,dtype", [((2, 32, 4, 8, 64), torch.bfloat16),     # MFMA kernels
                                         ((1, 32, 16, 16, 64), torch.bfloat16),
                                         # N (H / 4) >= 256 at D = 16: one 16-slice depth chunk, the
                                         # 18-slice walk of the B = 32 trunk
                                         ((64, 32, 16, 16, 64), torch.bfloat16),
                                         ((1, 32, 7, 4, 64), torch.bfloat16),     # depth walk of 7 (+2 halo)
                                         ((2, 32, 2, 8, 64), torch.bfloat16),     # no 3k-2 chunk: conv3d_c32_fwd
                                         ((2, 16, 3, 5, 8), torch.float32),       # direct kernels
                                         ((2, 32, 4, 4, 64), torch.float32),
                                         ((1, 24, 3, 4, 8), torch.bfloat16)])
def test_conv3d_kernels_vs_torch(shape, dtype):
    g = torch.Generator().manual_seed(3)
    N, C, D, H, W = shape
    Co = 32 if C == 32 else 16
    x = torch.randn(shape, generator=g)
    w = torch.randn(Co, C, 3, 3, 3, generator=g) * 0.05
    b = torch.randn(Co, generator=g)
    res = torch.randn(N, Co, D, H, W, generator=g)
    cs, xb, y, rec = run_conv3d(x, w, b, res=res, dtype=dtype, stats=True)
    torch.cuda.synchronize()
    xr, wr, rr = rnd(x, dtype), rnd(w, dtype), rnd(res, dtype)
    ref = F.conv3d(xr, wr, b, 1, 1) + rr
    tol_rel, tol_abs = (1e-5, 1e-5) if dtype == torch.float32 else (4e-3, 1.6e-2)
    assert rel(y.float(), ref) < tol_rel
    assert maxd(y.float(), ref) <= tol_abs * ref.abs().max().item()
    if rec is not None:                            # fused BN partials == sums of the stored output
        part, nb, bp = rec
        assert nb * bp == N * D * H * W
        p = part.view(nb, 2, Co).double().sum(0).cpu()
        yf = y.double().cpu().permute(1, 0, 2, 3, 4).reshape(Co, -1)
        assert rel(p[0], yf.sum(1)) < 1e-5
        assert rel(p[1], (yf * yf).sum(1)) < 1e-5
    # backward: data and weight gradients of sum(y * gy)
    gy = torch.randn(N, Co, D, H, W, generator=g)
    gyb = gy.cuda().to(dtype).contiguous(memory_format=CL3)
    dx, dw, db = ops3d.conv3d_backward(cs, xb, gyb)
    torch.cuda.synchronize()
    xr.requires_grad_(True)
    wr.requires_grad_(True)
    bb = b.clone().requires_grad_(True)
    (F.conv3d(xr, wr, bb, 1, 1) * rnd(gy, dtype)).sum().backward()
    assert rel(dx.float(), xr.grad) < tol_rel
    assert maxd(dx.float(), xr.grad) <= tol_abs * xr.grad.abs().max().item()
    wtol = 1e-5 if dtype == torch.float32 else 1e-4        # fp32 accumulation either way
    assert rel(dw, wr.grad) < wtol
    assert rel(db, bb.grad) < wtol


@pytest.mark.parametrize("shape", [(2, 32, 2, 8, 16), (2, 32, 16, 8, 16), (1, 32, 16, 3, 5)])
def test_depth_split_round_trip(shape):
    """(2, 32, 16, 8, 16): the bf16 C=32/D=16 LDS-tiled kernel; (1, 32, 16, 3, 5): its ragged fallback."""
    n, c, d, hh, ww = shape
    g = torch.Generator().manual_seed(5)
    h = torch.randn(n, c * d, hh, ww, generator=g)
    for dt in (torch.float32, torch.bfloat16):
        hb = h.cuda().to(dt).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        fs = ops3d.DepthSplitFn.apply(hb, c, d, dt)
        assert torch.equal(fs.float().cpu(), h.to(dt).float().view(*shape))
        back = ops3d.DepthMergeFn.apply(fs, dt)
        assert torch.equal(back.float().cpu(), h.to(dt).float())
        gg = torch.randn(*shape, generator=g).cuda()
        fs.backward(gg)
        assert torch.equal(hb.grad.float().cpu(), gg.to(dt).float().cpu().view(n, c * d, hh, ww))


def _res3d_case(mode):
    gd = torch.load(os.path.join(GOLD, "afe3d.pt"), weights_only=True)["res3d"]
    torch.manual_seed(int(gd["seed"]))
    blk = fv.ResBlock3D(32, False).cuda().train().set_compute_dtype(mode)
    x = gd["x"].cuda().requires_grad_(True)
    y = blk(x)
    (y.float() * gd["g"].cuda()).sum().backward()
    torch.cuda.synchronize()
    return gd, blk, x, y


def test_resblock3d_fp32_matches_reference():
    gd, blk, x, y = _res3d_case(torch.float32)
    assert rel(y, gd["out"]) < 1e-4
    assert rel(x.grad, gd["dx"]) < 1e-4
    for k, p in blk.named_parameters():
        if k == "layers.0.layers.2.bias":
            assert maxd(p.grad, gd["grads"][k]) < 1e-3, k
        else:
            assert rel(p.grad, gd["grads"][k]) < 1e-4, k
    sd = blk.state_dict()
    for k, v in gd["buffers"].items():
        if v.is_floating_point():
            assert rel(sd[k], v) < 1e-5, k
        else:
            assert torch.equal(sd[k].cpu(), v), k
    blk.eval()
    with torch.no_grad():
        ye = blk(gd["x"].cuda())
    assert rel(ye, gd["out_eval"]) < 1e-4


def test_resblock3d_bf16_vs_reference():
    gd, blk, x, y = _res3d_case(torch.bfloat16)     # W = 64: the MFMA kernels
    ey, edx = rel(y, gd["out"]), rel(x.grad, gd["dx"])
    ew = max(rel(p.grad, gd["grads"][k]) for k, p in blk.named_parameters() if k != "layers.0.layers.2.bias")
    print(f"\nResBlock3D bf16 vs reference: out {ey:.2e} dx {edx:.2e} max param grad {ew:.2e}")
    assert ey < 2e-2 and edx < 3e-2 and ew < 5e-2


def test_afe3d_fp32_matches_reference():
    gd = torch.load(os.path.join(GOLD, "afe3d.pt"), weights_only=True)["afe3d"]
    torch.manual_seed(int(gd["seed"]))
    afe = fv.AFE(False, [16, 32], n_res=1, C=32, D=2).cuda().train().set_compute_dtype(torch.float32)
    y = afe(gd["x"].cuda())
    assert y.shape == gd["out"].shape
    (y.float() * gd["g"].cuda()).sum().backward()
    torch.cuda.synchronize()
    assert rel(y, gd["out"]) < 1e-4
    dead = {"in_conv.layers.0.bias", "down.0.layers.0.layers.0.bias", "res.0.layers.0.layers.2.bias"}
    for k, p in afe.named_parameters():
        if k in dead:
            continue
        assert rel(p.grad, gd["grads"][k]) < 1e-3, k


@pytest.mark.parametrize("mode", [torch.float32, torch.bfloat16])
def test_afe_batched_conv3d_weight_prep_is_identical(mode, monkeypatch):
    """AFE.forward prepares every ResBlock3D conv's weight layouts in one launch
    (W3PrepBatch); the output and every gradient equal the per-conv preparation bit for bit
    (bf16 at W = 64: the MFMA layouts; fp32: the direct kernels' layouts)."""
    torch.manual_seed(3)
    afe = fv.AFE(False, [16, 32], n_res=2, C=32, D=4).cuda().train().set_compute_dtype(mode)
    x = torch.rand(1, 3, 128, 128, device="cuda")     # 3-D trunk [1, 32, 4, 64, 64]

    def run():
        for p in afe.parameters():
            p.grad = None
        y = afe(x)
        (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        torch.cuda.synchronize()
        return y.detach().clone(), {k: p.grad.clone() for k, p in afe.named_parameters() if p.grad is not None}

    sd = {k: v.clone() for k, v in afe.state_dict().items()}
    y1, g1 = run()
    assert afe.__dict__["_w3b"].bufs, "the batched preparation did not run"
    afe.load_state_dict(sd)
    monkeypatch.setattr(ops3d.W3PrepBatch, "prep", lambda self, d, device: None)
    for c in afe.modules():
        c.__dict__.pop("_c3prep", None)
    y2, g2 = run()
    assert torch.equal(y1, y2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_resblock3d_bf16_full_shape_vs_oracle():
    """One ResBlock3D at the AFE trunk's real shape (C=32, D=16, 64x64; one image) on the MFMA
    kernels against the fp32 CPU oracle on the same weights and input."""
    torch.manual_seed(7)
    blk = fv.ResBlock3D(32, False)
    sd = O.prepare_state({f"b.{k}": v for k, v in blk.state_dict().items()})
    blk = blk.cuda().train().set_compute_dtype(torch.bfloat16)
    g = torch.Generator().manual_seed(8)
    x = torch.randn(1, 32, 16, 64, 64, generator=g)
    gy = torch.randn(1, 32, 16, 64, 64, generator=g)
    xc = x.cuda().requires_grad_(True)
    y = blk(xc)
    (y.float() * gy.cuda()).sum().backward()
    torch.cuda.synchronize()
    xo = x.clone().requires_grad_(True)
    yo = O.res_block_3d(sd, "b", xo, True)
    (yo * gy).sum().backward()
    ey, edx = rel(y, yo), rel(xc.grad, xo.grad)
    ew = {k: rel(p.grad, sd["b." + k].grad) for k, p in blk.named_parameters() if k != "layers.0.layers.2.bias"}
    print(f"\nResBlock3D [1,32,16,64,64] bf16 vs oracle: out {ey:.2e} dx {edx:.2e} param grads "
          + " ".join(f"{k}={v:.1e}" for k, v in ew.items()))
    # BN affine gradients sum g * yhat over 65536 voxels of bf16-stored operands: looser
    assert ey < 2e-2 and edx < 3e-2
    for k, v in ew.items():
        assert v < (1e-1 if ".layers.0.weight" in k or ".layers.0.bias" in k else 5e-2), (k, v)
