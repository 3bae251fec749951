"""Pin the CPU oracle (oracle/facevae_cpu.py) against fixtures produced by the reference.

CPU only.  The fixtures come from tests/golden/make_golden.py (reference classes imported
from /root/reference in the build container).
"""
import os

import pytest
import torch
import torch.nn.functional as F

from oracle import facevae_cpu as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return torch.load(os.path.join(GOLD, name), weights_only=True)


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def dead_bias_keys(cfg):
    """Conv biases that feed a training-mode BN: their gradient is rounding noise (SURVEY.md
    Appendix A.6), so Adam moves them by ~±lr in a noise-determined direction.  They cannot
    change any output; compared with an absolute tolerance of 2*lr per step."""
    keys = set()
    for s in O.conv_specs(cfg):
        if s.block == "cna" or (s.block == "nac" and ".layers.0.layers.2" in s.prefix):
            keys.add(s.prefix + ".bias")
    return keys


def dead_bn_keys(cfg):
    """running_mean keys of the BNs that normalise a dead-bias conv's output (CNA: the block's
    own BN, `P.layers.0` conv -> `P.layers.1`; ResBlock conv1 `R.layers.0.layers.2` -> the second
    NAC's BN `R.layers.1.layers.0`)."""
    keys = set()
    for k in dead_bias_keys(cfg):
        p = k[:-len(".bias")]
        if p.endswith(".layers.0.layers.2"):
            keys.add(p[:-len(".layers.0.layers.2")] + ".layers.1.layers.0.running_mean")
        else:
            assert p.endswith(".layers.0"), p
            keys.add(p[:-len(".0")] + ".1.running_mean")
    return keys


def check_state(sd, ref, cfg, steps, tol):
    dead = dead_bias_keys(cfg)
    dead_bn = dead_bn_keys(cfg)
    assert dead_bn <= set(ref), sorted(dead_bn - set(ref))
    for k, v in ref.items():
        a = sd[k].detach()
        if not v.is_floating_point():
            assert torch.equal(a, v), k
        elif k in dead:
            assert (a - v).abs().max().item() <= 2 * cfg.lr * steps + 1e-7, k
        elif k in dead_bn:
            # the batch mean of a conv output carries that conv's (dead) bias, which Adam moves
            # by up to ±lr per step in a rounding-noise direction (above); the running mean takes
            # momentum (0.1) of it per step: |delta| <= 0.1 * 2 * lr * steps on top of rel < tol
            # (seen at 2.5e-5 relative on another host CPU's summation order)
            assert rel(a, v) < tol or (a - v).abs().max().item() <= 0.2 * cfg.lr * steps + 1e-7, k
        else:
            assert rel(a, v) < tol, k


def test_init_matches_reference_construction():
    g = load("toy_step.pt")
    sd = O.init_state(O.OracleConfig.toy(), seed=0)
    assert set(sd) == set(g["init"])
    for k in sd:
        assert torch.equal(sd[k], g["init"][k]), k


def test_full_init_checksums():
    g = load("full256.pt")
    sd = O.init_state(O.OracleConfig(), seed=0)
    assert set(sd) == set(g["init_checksums"])
    for k, v in sd.items():
        s = torch.tensor([v.double().sum().item(), v.double().abs().sum().item()], dtype=torch.float64)
        assert torch.allclose(s, g["init_checksums"][k].double(), rtol=1e-12, atol=1e-9), k


def test_toy_step_matches_reference():
    g = load("toy_step.pt")
    cfg = O.OracleConfig.toy()
    sd = O.prepare_state(g["init"])
    opt = O.adam_init(sd)
    out, grads = O.train_step(sd, opt, g["x"], g["eps"], cfg)
    s1 = g["step1"]
    assert rel(out["y"], s1["y"]) < 1e-6
    assert rel(out["mu"], s1["mu"]) < 1e-6
    assert abs(out["R"].item() - s1["R"].item()) <= 1e-6 * abs(s1["R"].item())
    assert abs(out["K"].item() - s1["K"].item()) <= 1e-6 * abs(s1["K"].item())
    dead = dead_bias_keys(cfg)
    for k, gr in s1["grads"].items():
        if k in dead:
            assert (grads[k] - gr).abs().max().item() < 1e-6, k
        else:
            assert rel(grads[k], gr) < 1e-5, k
    check_state(sd, s1["state"], cfg, 1, 1e-6)
    # steps 2, 3
    Rs, Ks = [out["R"].item()], [out["K"].item()]
    for _ in range(2):
        o, _ = O.train_step(sd, opt, g["x"], g["eps"], cfg)
        Rs.append(o["R"].item())
        Ks.append(o["K"].item())
    assert torch.allclose(torch.tensor(Rs, dtype=torch.float64), g["step3"]["R"].double(), rtol=1e-5)
    assert torch.allclose(torch.tensor(Ks, dtype=torch.float64), g["step3"]["K"].double(), rtol=1e-5)
    assert rel(o["y"], g["step3"]["y"]) < 1e-5
    check_state(sd, g["step3"]["state"], cfg, 3, 1e-5)


def test_full256_two_steps_match_reference():
    g = load("full256.pt")
    cfg = O.OracleConfig()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    sd = O.prepare_state(O.init_state(cfg, 0))
    opt = O.adam_init(sd)
    B = 2
    x = torch.rand(B, 3, 256, 256, generator=torch.Generator().manual_seed(1234))
    eps = torch.randn(B, 256, 64, 64, generator=torch.Generator().manual_seed(1235))
    o1, _ = O.train_step(sd, opt, x, eps, cfg)
    o2, _ = O.train_step(sd, opt, x, eps, cfg)
    assert torch.allclose(torch.stack([o1["R"], o2["R"]]).double(), g["R"].double(), rtol=1e-5)
    assert torch.allclose(torch.stack([o1["K"], o2["K"]]).double(), g["K"].double(), rtol=1e-5)
    assert rel(o1["y"][:, :, ::17, ::13], g["y1_samples"]) < 1e-5


BLOCKS = ["cna_relu", "cna_leaky_sn", "cna_7x7", "down", "up_sn", "res_sn", "same"]
# per block: the conv biases that feed a training-mode BN (prefix '' = the block; see oracle_block)
BLOCK_DEAD_BIAS = {"cna_relu": {"layers.0.bias"}, "cna_leaky_sn": {"layers.0.bias"}, "cna_7x7": {"layers.0.bias"},
                   "down": {"layers.0.layers.0.bias"}, "up_sn": {"layers.1.layers.0.bias"},
                   "res_sn": {"layers.0.layers.2.bias"}, "same": {"layers.layers.0.bias"}}


def oracle_block(name, sd, x):
    """Each reference block restated with the oracle primitives (prefix '' -> 'layers')."""
    sd = {"m." + k: v for k, v in sd.items()}
    if name == "cna_relu" or name == "cna_7x7":
        return O.conv_block(sd, "m", x, "CNA", True), sd
    if name == "same":                                   # SameBlock2D.layers is the ConvBlock2D
        return O.conv_block(sd, "m.layers", x, "CNA", True), sd
    if name == "cna_leaky_sn":
        return O.conv_block(sd, "m", x, "CNA", True, "leakyrelu"), sd
    if name == "down":
        return F.avg_pool2d(O.conv_block(sd, "m.layers.0", x, "CNA", True), 2), sd
    if name == "up_sn":
        return O.conv_block(sd, "m.layers.1", F.interpolate(x, scale_factor=2.0), "CNA", True), sd
    if name == "res_sn":
        t = O.conv_block(sd, "m.layers.0", x, "NAC", True)
        return x + O.conv_block(sd, "m.layers.1", t, "NAC", True), sd
    raise KeyError(name)


@pytest.mark.parametrize("name", BLOCKS)
def test_block_cases(name):
    c = load("blocks.pt")[name]
    sd = O.prepare_state(c["init"])
    x = c["x"].clone().requires_grad_(True)
    y, sdp = oracle_block(name, sd, x)
    assert rel(y, c["y"]) < 1e-6
    (y * c["gy"]).sum().backward()
    assert rel(x.grad, c["gx"]) < 1e-5
    gscale = max(gr.abs().max().item() for gr in c["grads"].values())
    dead = BLOCK_DEAD_BIAS[name]
    for k, gr in c["grads"].items():
        g = sdp["m." + k].grad
        if k in dead:
            # a conv bias feeding a training-mode BN (dead_bias_keys): its gradient is rounding
            # noise whose digits follow the host CPU's summation order -- absolute bound only
            assert gr.abs().max().item() < 1e-4 * gscale, k
            assert (g - gr).abs().max().item() <= 1e-4 * gscale, k
        else:
            assert rel(g, gr) < 1e-5, k
    for k, v in c["state"].items():
        if v.is_floating_point():
            assert rel(sdp["m." + k].detach(), v) < 1e-6, k


CONVT_CASES = {
    "demod_leaky": (6, 8, 4, 2, 1, "demod", None, 0.2),
    "plain_untied": (4, 8, 4, 2, 1, None, (10, 12), None),
    "demod_relu_k3s1": (5, 8, 3, 1, 1, "demod", None, 0.0),
}


@pytest.mark.parametrize("name", list(CONVT_CASES))
def test_convt_elr_oracle_matches_reference(name):
    """ConvTranspose2dELR restatement (oracle.convt_elr) vs the reference module's forward /
    backward (tests/golden/make_golden_convt.py)."""
    g = load("convt_elr.pt")[name]
    inch, outch, k, s, p, norm, ub, slope = CONVT_CASES[name]
    gain = O.convt_elr_gain(inch, k, s, norm, slope)
    assert abs(gain - g["weightgain"].item()) < 1e-12
    w = g["weight"].clone().requires_grad_(True)
    b = g["bias"].clone().requires_grad_(True)
    x = g["x"].clone().requires_grad_(True)
    y = O.convt_elr(x, w, b, s, p, norm, gain, slope)
    y.backward(g["g"])
    assert rel(y.detach(), g["y"]) < 1e-6
    assert rel(x.grad, g["dx"]) < 1e-6
    assert rel(w.grad, g["dweight"]) < 1e-5
    assert rel(b.grad, g["dbias"]) < 1e-6


def test_convt_elr_module_init_matches_reference():
    """The product module draws the reference's init (blockinit of one randn) and gain."""
    import fvamd  # noqa: F401
    import facevae_amd as fv
    gold = load("convt_elr.pt")
    for i, (name, (inch, outch, k, s, p, norm, ub, slope)) in enumerate(CONVT_CASES.items()):
        act = None if slope is None else (torch.nn.ReLU() if slope == 0.0 else torch.nn.LeakyReLU(slope))
        torch.manual_seed(100 + i)
        m = fv.ConvTranspose2dELR(inch, outch, k, s, p, norm=norm, ub=ub, act=act)
        assert torch.equal(m.weight.detach(), gold[name]["weight"]), name
        assert m.bias.shape == gold[name]["bias"].shape
        assert abs(m.weightgain - gold[name]["weightgain"].item()) < 1e-12
    torch.manual_seed(0)
    m = fv.ConvTranspose2dELR(64, 64, 4, 2, 1, norm="demod")
    assert torch.equal(m.weight.detach()[0, 0], gold["gpu_init"]["weight_00"])
    assert abs(m.weight.double().sum().item() - gold["gpu_init"]["sum"].item()) < 1e-9


MOD_CASES = {
    "mod_demod_leaky": (6, 8, 4, 2, 1, "demod", 5, 0.2),
    "mod_plain_k3s1": (5, 8, 3, 1, 1, None, 4, None),
}


@pytest.mark.parametrize("name", list(MOD_CASES))
def test_convt_elr_modulated_oracle_matches_reference(name):
    """Modulated ConvTranspose2dELR restatement (oracle.convt_elr_mod) vs the reference module."""
    g = load("convt_elr.pt")[name]
    inch, outch, k, s, p, norm, wsize, slope = MOD_CASES[name]
    gain = O.convt_elr_gain(inch, k, s, norm, slope)
    assert abs(gain - g["weightgain"].item()) < 1e-12
    assert abs(1.0 / wsize ** 0.5 - g["affine_gain"].item()) < 1e-12
    prm = {kk: v.clone().requires_grad_(True) for kk, v in g["init"].items()}
    x, w = g["x"].clone().requires_grad_(True), g["w"].clone().requires_grad_(True)
    y = O.convt_elr_mod(x, w, prm["weight"], prm["bias"], prm["affine.weight"], prm["affine.bias"],
                        g["affine_gain"].item(), s, p, norm, gain, slope)
    y.backward(g["g"])
    assert rel(y.detach(), g["y"]) < 1e-6
    assert rel(x.grad, g["dx"]) < 1e-5 and rel(w.grad, g["dw"]) < 1e-5
    for kk, v in g["grads"].items():
        assert rel(prm[kk].grad, v) < 1e-5, kk


def test_convt_elr_modulated_module_init_matches_reference():
    import fvamd  # noqa: F401
    import facevae_amd as fv
    for j, (name, (inch, outch, k, s, p, norm, wsize, slope)) in enumerate(MOD_CASES.items()):
        g = load("convt_elr.pt")[name]
        act = None if slope is None else torch.nn.LeakyReLU(slope)
        torch.manual_seed(500 + j)
        m = fv.ConvTranspose2dELR(inch, outch, k, s, p, wsize=wsize, norm=norm, act=act)
        sd = m.state_dict()
        assert set(sd) == set(g["init"])
        for kk in ("weight", "affine.weight"):
            assert torch.equal(sd[kk], g["init"][kk]), (name, kk)
