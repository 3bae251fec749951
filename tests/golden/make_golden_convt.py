"""Golden fixtures for ConvTranspose2dELR (models_utils.py:404-516), FROM THE REFERENCE.

Build container only (needs /root/reference):  python tests/golden/make_golden_convt.py

Imports the reference `models_utils.py` read-only, constructs ConvTranspose2dELR under fixed
seeds, runs forward + backward on seeded inputs and stores plain tensors in convt_elr.pt
(loaded with weights_only=True): init weight, input, upstream gradient, output, input /
weight / bias gradients per case, and the init-weight checksums of the GPU-test shape.
"""
import os
import sys

import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = {
    # name: (inch, outch, k, s, p, norm, ub, act_slope, x shape)
    "demod_leaky": (6, 8, 4, 2, 1, "demod", None, 0.2, (2, 6, 5, 7)),
    "plain_untied": (4, 8, 4, 2, 1, None, (10, 12), None, (1, 4, 5, 6)),
    "demod_relu_k3s1": (5, 8, 3, 1, 1, "demod", None, 0.0, (2, 5, 6, 6)),
}
MOD_CASES = {
    # name: (inch, outch, k, s, p, norm, wsize, act_slope, x shape)
    "mod_demod_leaky": (6, 8, 4, 2, 1, "demod", 5, 0.2, (2, 6, 5, 7)),
    "mod_plain_k3s1": (5, 8, 3, 1, 1, None, 4, None, (3, 5, 6, 6)),
}
GPU_SHAPE = (64, 64, 4, 2, 1, "demod")    # tests/test_kernels_gpu.py::test_conv_transpose_elr


def main():
    sys.path.insert(0, REF)
    import models_utils as MU  # noqa: E402  (reference, read-only)
    nn = torch.nn
    out = {}
    for i, (name, (inch, outch, k, s, p, norm, ub, slope, xs)) in enumerate(CASES.items()):
        act = None if slope is None else (nn.ReLU() if slope == 0.0 else nn.LeakyReLU(slope))
        torch.manual_seed(100 + i)
        m = MU.ConvTranspose2dELR(inch, outch, k, s, p, norm=norm, ub=ub, act=act)
        with torch.no_grad():
            m.bias.normal_(generator=torch.Generator().manual_seed(200 + i))
        w0, b0 = m.weight.detach().clone(), m.bias.detach().clone()
        x = torch.randn(*xs, generator=torch.Generator().manual_seed(300 + i)).requires_grad_(True)
        y = m(x)
        g = torch.randn(y.shape, generator=torch.Generator().manual_seed(400 + i))
        y.backward(g)
        out[name] = {"weight": w0, "bias": b0, "x": x.detach(), "g": g, "y": y.detach(), "dx": x.grad,
                     "dweight": m.weight.grad, "dbias": m.bias.grad,
                     "weightgain": torch.tensor(m.weightgain, dtype=torch.float64)}
    # per-sample affine modulation (wsize > 0, forward(x, w)): models_utils.py:444-446, 486-495
    for j, (name, (inch, outch, k, s, p, norm, wsize, slope, xs)) in enumerate(MOD_CASES.items()):
        act = None if slope is None else nn.LeakyReLU(slope)
        torch.manual_seed(500 + j)
        m = MU.ConvTranspose2dELR(inch, outch, k, s, p, wsize=wsize, norm=norm, act=act)
        with torch.no_grad():
            m.bias.normal_(generator=torch.Generator().manual_seed(600 + j))
            m.affine.bias.normal_(generator=torch.Generator().manual_seed(610 + j))
        init = {kk: v.detach().clone() for kk, v in m.state_dict().items()}
        x = torch.randn(*xs, generator=torch.Generator().manual_seed(700 + j)).requires_grad_(True)
        wv = torch.randn(xs[0], wsize, generator=torch.Generator().manual_seed(710 + j)).requires_grad_(True)
        y = m(x, wv)
        g = torch.randn(y.shape, generator=torch.Generator().manual_seed(720 + j))
        y.backward(g)
        out[name] = {"init": init, "x": x.detach(), "w": wv.detach(), "g": g, "y": y.detach(), "dx": x.grad,
                     "dw": wv.grad, "grads": {kk: v.grad.clone() for kk, v in m.named_parameters()},
                     "weightgain": torch.tensor(m.weightgain, dtype=torch.float64),
                     "affine_gain": torch.tensor(m.affine.weightgain, dtype=torch.float64)}
    inch, outch, k, s, p, norm = GPU_SHAPE
    torch.manual_seed(0)
    m = MU.ConvTranspose2dELR(inch, outch, k, s, p, norm=norm)
    out["gpu_init"] = {"sum": m.weight.detach().double().sum(), "abs_sum": m.weight.detach().double().abs().sum(),
                       "weight_00": m.weight.detach()[0, 0].clone()}
    torch.save(out, os.path.join(HERE, "convt_elr.pt"))
    print("wrote convt_elr.pt:", list(out))


if __name__ == "__main__":
    main()
