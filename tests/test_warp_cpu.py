"""Warp path on the CPU: the oracle restatement against fixtures generated
from the reference's utils.py / MFE tail / Generator (tests/golden/make_golden_warp.py)."""
import os

import torch

from oracle import facevae_cpu as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load():
    return torch.load(os.path.join(GOLD, "warp.pt"), weights_only=True)


def rel(a, b):
    return ((a.detach().double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def test_motion_functions_match_reference():
    m = load()["motion"]
    ins = [m[k].clone().requires_grad_(True) for k in ("fs", "kp_s", "kp_d", "Rs", "Rd")]
    sm = O.sparse_motions(*ins)
    hm = O.heatmap_representations(ins[0], ins[1], ins[2])
    ds = O.deformed_source(ins[0], sm)
    assert rel(sm, m["sm"]) < 1e-6 and rel(hm, m["hm"]) < 1e-6 and rel(ds, m["ds"]) < 1e-6
    ((sm * m["g_sm"]).sum() + (hm * m["g_hm"]).sum() + (ds * m["g_ds"]).sum()).backward()
    for n, t in zip(("fs", "kp_s", "kp_d", "Rs", "Rd"), ins):
        assert rel(t.grad, m["grads"][n]) < 1e-5, n


def test_motion_mask_matches_reference():
    m = load()["mask"]
    lt, st = m["logits"].clone().requires_grad_(True), m["sm"].clone().requires_grad_(True)
    d, mask = O.motion_mask(lt, st)
    assert rel(d, m["deformation"]) < 1e-6 and rel(mask, m["mask"]) < 1e-6
    ((d * m["g_def"]).sum() + (mask * m["g_mask"]).sum()).backward()
    assert rel(lt.grad, m["d_logits"]) < 1e-5 and rel(st.grad, m["d_sm"]) < 1e-5


def test_generator_warp_matches_reference():
    g = load()["generator"]
    sd = O.prepare_state({f"generator.{k}": v for k, v in g["init"].items()})
    ins = [g[k].clone().requires_grad_(True) for k in ("fs", "deformation", "occlusion")]
    y = O.generator_warp(sd, *ins, n_res=1, n_up=1, training=True)
    assert rel(y, g["out"]) < 1e-5
    (y * g["g"]).sum().backward()
    for n, t in zip(("d_fs", "d_deformation", "d_occlusion"), ins):
        assert rel(t.grad, g[n]) < 1e-4, n
    for k, v in g["grads"].items():
        if k == "in_conv.layers.0.bias" or k.endswith("layers.0.layers.2.bias") or k == "up.0.layers.1.layers.0.bias":
            continue                                # biases feeding a training-mode BN (rounding noise)
        assert rel(sd["generator." + k].grad, v) < 1e-4, k
