"""Probe: internal accumulation precision of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3):
rows of one large product and many small ones, against the exact sum."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fvamd  # noqa: E402,F401
from facevae_amd import _lib as L  # noqa: E402


def probe(a, b):
    ac = a.to(torch.float8_e4m3fn).view(torch.uint8).cuda()
    bc = b.to(torch.float8_e4m3fn).view(torch.uint8).cuda()
    c = torch.empty(16, 16, device="cuda")
    L.call("fv_fp8_mfma_probe", ac.data_ptr(), bc.data_ptr(), c.data_ptr(), L.stream())
    torch.cuda.synchronize()
    ref = a.to(torch.float8_e4m3fn).double() @ b.to(torch.float8_e4m3fn).double().t()
    return c.double().cpu(), ref


ones = torch.ones(16, 128)
for big in (448.0, 64.0, 8.0, 1.0):
    for small in (2.0 ** -9, 2.0 ** -6, 2.0 ** -3, 0.5):
        a = torch.full((16, 128), small)
        a[:, 0] = big
        c, ref = probe(a, ones)
        print(f"big {big:6g} + 127 x {small:.6g}: mfma {c[0, 0].item():.9g} exact {ref[0, 0].item():.9g} "
              f"diff {c[0, 0].item() - ref[0, 0].item():+.3e}")
# one small term at each position, the big one elsewhere
a = torch.zeros(16, 128)
a[:, 5] = 448.0
for i in range(16):
    a[i, 64 + i] = 2.0 ** -9 * (i + 1) if i < 7 else 2.0 ** -6 * (i - 6)
c, ref = probe(a, ones)
print("single small term rows:", [(round(c[i, 0].item() - 448.0, 9), round(ref[i, 0].item() - 448.0, 9)) for i in range(16)])
# sign mix: +big, -big, small terms
a = torch.full((16, 128), 2.0 ** -7)
a[:, 0] = 448.0
a[:, 1] = -448.0
c, ref = probe(a, ones)
print(f"+448 -448 + 126 x 2^-7: mfma {c[0, 0].item():.9g} exact {ref[0, 0].item():.9g}")
# random heavy-tailed rows
g = torch.Generator().manual_seed(0)
a = torch.randn(16, 128, generator=g) ** 3 * 4
c, ref = probe(a, ones)
print("heavy rows rel err:", ((c[:, 0] - ref[:, 0]).abs() / ref.abs().sum(1).clamp_min(1e-30) * 0 + (c[:, 0] - ref[:, 0]).abs()).tolist()[:6])
