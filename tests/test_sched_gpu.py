"""SIMD-partner schedules of the linear-halo 3x3 kernels (conv.hip conv3_halo_fwd3 SCH,
FV_RES_SCHED = 0..3): static priority and the half-step stagger reorder instructions only, so
every schedule must give bit-identical forward / data-gradient outputs, and the default one
must match torch fp32 at the bf16 tolerance of tests/test_kernels_gpu.py.  Shapes: the
ResBlock2D conv (256 -> 256, 256-channel co tile) and a 128-channel co tile."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
from facevae_amd import _lib as L  # noqa: E402
from facevae_amd import ops  # noqa: E402

from test_kernels_gpu import conv_setup, gen, rel  # noqa: E402

CL = torch.channels_last
CASES = [
    # N, cin, cout, H, W
    (2, 256, 256, 16, 64),
    (1, 256, 256, 8, 128),
    (2, 64, 128, 8, 64),
    (4, 128, 128, 12, 64),
    (2, 128, 64, 16, 64),      # the 64-co tile (AFE.down1's data gradient shape)
]


def _run(case, sched, monkeypatch, pers_grid=None):
    N, cin, cout, H, W = case
    monkeypatch.setenv("FV_RES_SCHED", str(sched))
    if pers_grid is None:
        monkeypatch.delenv("FV_PERS_GRID", raising=False)
    else:
        monkeypatch.setenv("FV_PERS_GRID", str(pers_grid))
    g = gen(300 + cin + H)
    x = torch.randn(N, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    b = torch.randn(cout, generator=g)
    gy = torch.randn(N, cout, H, W, generator=g)
    d, xb, wk, wt, shp = conv_setup(x, w, 3, torch.bfloat16, need_wt=True)
    y = torch.empty(shp, dtype=torch.bfloat16, device="cuda", memory_format=CL)
    nb = L.query("fv_conv2d_stats_blocks", ctypes.byref(d))
    part = torch.empty(nb * 2 * cout, device="cuda")
    L.call("fv_conv2d_fwd", ctypes.byref(d), xb.data_ptr(), wk.data_ptr(), b.cuda().data_ptr(), None, None, None,
           y.data_ptr(), part.data_ptr(), L.stream())
    gyb = gy.cuda().to(torch.bfloat16).contiguous(memory_format=CL)
    dx = torch.empty((N, cin, H, W), dtype=torch.bfloat16, device="cuda", memory_format=CL)
    L.call("fv_conv2d_bwd_data", ctypes.byref(d), gyb.data_ptr(), cout, wt.data_ptr(), dx.data_ptr(), L.stream())
    torch.cuda.synchronize()
    return x, w, b, gy, y.float().cpu(), part.cpu(), dx.float().cpu()


@pytest.mark.parametrize("case", CASES)
def test_res_schedules_bit_identical(case, monkeypatch):
    x, w, b, gy, y0, p0, dx0 = _run(case, 0, monkeypatch)
    xr = x.clone().requires_grad_(True)
    ref = F.conv2d(xr, w, b, padding=1)
    (ref * gy).sum().backward()
    assert rel(y0, ref.detach()) < 3e-2
    assert rel(dx0, xr.grad) < 3e-2
    for s in (1, 2, 3):
        _, _, _, _, y, p, dx = _run(case, s, monkeypatch)
        assert torch.equal(y, y0), f"schedule {s}: forward differs"
        assert torch.equal(p, p0), f"schedule {s}: BN records differ"
        assert torch.equal(dx, dx0), f"schedule {s}: data gradient differs"
    # persistent tiles (FV_PERS_GRID: a grid of 3 blocks walks every tile, the next tile's
    # prologue DMA issued under the previous epilogue's stores): the same bits
    for s in (0, 2):
        _, _, _, _, y, p, dx = _run(case, s, monkeypatch, pers_grid=3)
        assert torch.equal(y, y0) and torch.equal(p, p0) and torch.equal(dx, dx0), f"persistent, schedule {s}"

