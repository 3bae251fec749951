"""BN-apply + ReLU of AFE.in_conv in down1's operand staging (ops.CNAPairFn, VERDICT r4 item 5
"option B"): conv3c64_fwd<true> transforms the pre-BN rows in LDS with act_fwd's arithmetic and
the sliding-row weight gradient's PRO variant does the same, so forward output, BN statistics,
running statistics and every parameter gradient must be BIT-IDENTICAL to the unfused chain
(ConvBNActFn twice: act_fwd pass + plain kernels) on the same inputs.  Shapes: the bench's AFE 2-D
trunk (3 -> 64 -> 128 -> 256) at 64x64 and at 256x256, B=2."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import ops  # noqa: E402


def _run(m, x, g, fused):
    prev = ops._BN_PRO
    ops._BN_PRO = fused
    try:
        m = copy.deepcopy(m)
        assert ops.bn_pro_pair_ok(m.in_conv, m.down[0].layers[0], x) == fused
        h = m.forward_2d(x)
        (h.float() * g).sum().backward()
        torch.cuda.synchronize()
    finally:
        ops._BN_PRO = prev
    grads = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters() if p.grad is not None}
    state = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    return h.detach().float().cpu(), grads, state


@pytest.mark.parametrize("H", [64, 256])
def test_cna_pair_bit_identical(H):
    torch.manual_seed(0)
    m = fv.models.AFE(False, [64, 128, 256], 0, C=32, D=1).cuda().train().set_compute_dtype(torch.bfloat16)
    x = torch.rand(2, 3, H, H, generator=torch.Generator().manual_seed(5)).cuda()
    g = torch.randn(2, 32, H // 4, H // 4, generator=torch.Generator().manual_seed(6)).cuda()
    h0, g0, s0 = _run(m, x, g, False)
    h1, g1, s1 = _run(m, x, g, True)
    assert torch.equal(h0, h1), (h0 - h1).abs().max()
    assert g0.keys() == g1.keys() and len(g0) >= 12
    for k in g0:
        assert torch.equal(g0[k], g1[k]), (k, (g0[k] - g1[k]).abs().max())
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
