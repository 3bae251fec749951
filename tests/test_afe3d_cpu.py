"""AFE 3-D trunk on the CPU: the oracle restatement (oracle.res_block_3d /
encode_afe) against fixtures generated from the reference ResBlock3D / AFE
(tests/golden/make_golden_3d.py), and the product modules' constructors against the
reference's initial parameters (same RNG draws, same state-dict keys)."""
import os

import torch

import fvamd  # noqa: F401
import facevae_amd as fv
from oracle import facevae_cpu as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load():
    return torch.load(os.path.join(GOLD, "afe3d.pt"), weights_only=True)


def rel(a, b):
    return ((a.detach().double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def build_state(module, init_sum, prefix):
    """state dict of a freshly built product module, checked against the reference init."""
    sd = module.state_dict()
    for k, v in init_sum.items():
        assert abs(sd[k].double().sum().item() - v.item()) <= 1e-9 * (1 + abs(v.item())), k
    assert set(k for k, v in sd.items() if v.is_floating_point()) == set(init_sum)
    return O.prepare_state({f"{prefix}.{k}": v for k, v in sd.items()})


def test_res3d_oracle_matches_reference():
    g = load()["res3d"]
    torch.manual_seed(int(g["seed"]))
    sd = build_state(fv.ResBlock3D(32, False), g["init_sum"], "b")
    x = g["x"].clone().requires_grad_(True)
    y = O.res_block_3d(sd, "b", x, True)
    (y * g["g"]).sum().backward()
    assert rel(y, g["out"]) < 1e-6
    assert rel(x.grad, g["dx"]) < 1e-5
    for k, v in g["grads"].items():
        a = sd["b." + k].grad
        if k == "layers.0.layers.2.bias":      # feeds a training-mode BN: rounding noise
            assert (a - v).abs().max().item() < 1e-3, k
        else:
            assert rel(a, v) < 1e-5, k
    for k, v in g["buffers"].items():
        if v.is_floating_point():
            assert rel(sd["b." + k], v) < 1e-6, k
        else:
            assert torch.equal(sd["b." + k], v), k
    with torch.no_grad():
        ye = O.res_block_3d(sd, "b", g["x"], False)
    assert rel(ye, g["out_eval"]) < 1e-6


def test_afe3d_oracle_matches_reference():
    g = load()["afe3d"]
    torch.manual_seed(int(g["seed"]))
    sd = build_state(fv.AFE(False, [16, 32], n_res=1, C=32, D=2), g["init_sum"], "afe")
    y = O.encode_afe(sd, g["x"], [16, 32], 32, 2, 1, True)
    (y * g["g"]).sum().backward()
    assert y.shape == g["out"].shape
    assert rel(y, g["out"]) < 1e-5
    dead = {"in_conv.layers.0.bias", "down.0.layers.0.layers.0.bias", "res.0.layers.0.layers.2.bias"}
    for k, v in g["grads"].items():
        a = sd["afe." + k].grad
        if k in dead:
            assert (a - v).abs().max().item() < 1e-2 * (1 + v.abs().max().item()), k
        else:
            assert rel(a, v) < 1e-4, k


def test_resblock3d_surface():
    blk = fv.ResBlock3D(32, False)
    keys = list(blk.state_dict())
    assert keys[:7] == ["layers.0.layers.0.weight", "layers.0.layers.0.bias", "layers.0.layers.0.running_mean",
                        "layers.0.layers.0.running_var", "layers.0.layers.0.num_batches_tracked",
                        "layers.0.layers.2.weight", "layers.0.layers.2.bias"]
    assert blk.state_dict()["layers.0.layers.2.weight"].shape == (32, 32, 3, 3, 3)
