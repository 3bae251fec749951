"""Every caller-sized buffer the product allocates stays inside its queried size (VERDICT r5
weak item 10: two faults in two rounds came from a buffer sized apart from the tile plan that
writes it -- the r4 weight image, the r5 BN records).

`ops._empty` is the one allocator of the product's caller-sized buffers -- weight-gradient
split slabs and bias slabs (incl. the sub-pixel and packed 7x7 layouts), BN statistics
records, store-pass records, fold scratch, spectral-norm / fp8 / loss / reparameterisation
workspaces, the grid-sample bucket workspace (warp.py) and the conv3d weight-gradient
workspace (ops3d.py).  Here it hands out each buffer with a 4 KB guard region of a sentinel
byte behind it; a whole training step runs (forward, backward, Adam: every launch of the
timed step at 2 images) and every guard must come back untouched.  The §8(f) kernels (grid
sample input gradient incl. a collapsed grid, a ResBlock3D forward / backward) are checked
the same way."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import ops, warp  # noqa: E402

GUARD = 4096
SENT = 0xA5


class _Guarded:
    def __init__(self):
        self.bufs = []

    def __call__(self, n, dtype, device):
        n = int(n)
        es = torch.empty(0, dtype=dtype).element_size()
        raw = torch.full((n * es + GUARD,), SENT, dtype=torch.uint8, device=device)
        self.bufs.append((raw, n * es))
        return raw[:n * es].view(dtype)

    def check(self):
        torch.cuda.synchronize()
        bad = [(i, nb) for i, (raw, nb) in enumerate(self.bufs) if not bool((raw[nb:] == SENT).all())]
        return len(self.bufs), bad


@pytest.mark.parametrize("dtype_name", ["bfloat16", "float8_e4m3fn", "float32"])
def test_step_workspaces_stay_in_bounds(dtype_name, monkeypatch):
    g = _Guarded()
    monkeypatch.setattr(ops, "_empty", g)
    big = dtype_name != "float32"
    cfg = fv.FaceVAEConfig(H=256) if big else fv.FaceVAEConfig.toy()
    torch.manual_seed(0)
    m = fv.FaceVAE(cfg).cuda().train().set_compute_dtype(getattr(torch, dtype_name))
    opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
    gen = torch.Generator().manual_seed(3)
    x = torch.rand(2, 3, cfg.H, cfg.H, generator=gen).cuda()
    eps = torch.randn(2, cfg.latent, cfg.latent_hw, cfg.latent_hw, generator=gen).cuda()
    for _ in range(2):                    # the fp8 sites are seeded on the first step
        opt.zero_grad(set_to_none=True)
        y, mu, ls = m(x, eps)
        (cfg.w_R * fv.ReconLoss()((x, y)) + cfg.w_K * fv.KLDivergenceLoss()((mu, ls))).backward()
        opt.step()
    n, bad = g.check()
    assert n > 50, n                      # the step's workspaces went through the guard
    assert not bad, f"{len(bad)} of {n} buffers written past their queried size: {bad[:8]}"


@pytest.mark.parametrize("collapse", [False, True])
def test_grid_sample_workspace_stays_in_bounds(collapse, monkeypatch):
    g = _Guarded()
    monkeypatch.setattr(ops, "_empty", g)
    gen = torch.Generator().manual_seed(12)
    N, C, Di, Hi, Wi, Do, Ho, Wo = 2, 32, 4, 8, 16, 8, 16, 16
    inp = torch.randn(N, C, Di, Hi, Wi, generator=gen)
    grid = (torch.rand(N, Do, Ho, Wo, 3, generator=gen) - 0.5) * 2.2
    if collapse:
        grid = grid * 0.01 - 0.99
    for dt in (torch.float32, torch.bfloat16):
        xi = inp.cuda().to(dt).contiguous(memory_format=torch.channels_last_3d).requires_grad_(True)
        out = warp.GridSample3dFn.apply(xi, grid.cuda(), 1, dt)
        out.backward(torch.randn(out.shape, generator=gen).cuda().to(out.dtype))
    n, bad = g.check()
    assert n >= 2 and not bad, (n, bad)


def test_conv3d_workspaces_stay_in_bounds(monkeypatch):
    g = _Guarded()
    monkeypatch.setattr(ops, "_empty", g)
    torch.manual_seed(5)
    for mode in (torch.float32, torch.bfloat16):
        blk = fv.ResBlock3D(32, False).cuda().train().set_compute_dtype(mode)
        x = torch.randn(2, 32, 16, 32, 64).cuda().requires_grad_(True)
        y = blk(x)
        y.float().sum().backward()
    n, bad = g.check()
    assert n > 4 and not bad, (n, bad)
