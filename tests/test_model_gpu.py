"""GPU parity of the drop-in modules and of the full FaceVAE training step against fixtures
generated from the reference (tests/golden/*.pt) and against the CPU oracle at 256x256.

Tolerances (written here, as BASELINE.md §3 requires): fp32 mode (exact-fp32 MFMA) —
1e-4 relative L2 per tensor for blocks, and the north_star bar of 1e-3 relative for the
reconstructed image, KL and recon losses of the training step.  bf16 mode deviations are
measured and reported, and gated only loosely (they are not the parity gate).
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from oracle import facevae_cpu as O  # noqa: E402  (checker only)

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return torch.load(os.path.join(GOLD, name), weights_only=True)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


BLOCKS = {
    "cna_relu": lambda: fv.ConvBlock2D("CNA", 16, 32, 3, 1, 1, False),
    "cna_leaky_sn": lambda: fv.ConvBlock2D("CNA", 32, 32, 3, 1, 1, True, nonlinearity_type="leakyrelu"),
    "cna_7x7": lambda: fv.ConvBlock2D("CNA", 3, 16, 7, 1, 3, False),
    "down": lambda: fv.DownBlock2D(16, 32, False),
    "up_sn": lambda: fv.UpBlock2D(32, 16, True),
    "res_sn": lambda: fv.ResBlock2D(32, True),
    "same": lambda: fv.SameBlock2D(32, 64, False),
}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("name", list(BLOCKS))
def test_block_matches_reference(name, dtype):
    c = load("blocks.pt")[name]
    m = BLOCKS[name]()
    m.load_state_dict(c["init"])
    m = m.cuda().train().set_compute_dtype(dtype)
    x = c["x"].cuda().requires_grad_(True)
    y = m(x)
    (y.float() * c["gy"].cuda()).sum().backward()
    torch.cuda.synchronize()
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    assert rel(y.float(), c["y"]) < tol
    assert rel(x.grad, c["gx"]) < tol * 2
    named = dict(m.named_parameters())
    for k, g in c["grads"].items():
        if k.endswith("bias") and (g.abs().max() < 1e-4):      # dead bias before a BN
            # its gradient is rounding noise of sum(dy): ~1e-6 in fp32,
            # ~1e-2..1e-1 with bf16-stored dy; it cannot affect any output
            assert (named[k].grad.cpu() - g).abs().max() < (1e-3 if dtype == torch.float32 else 0.5)
        else:
            assert rel(named[k].grad, g) < tol * 2, k
    sd = m.state_dict()
    for k, v in c["state"].items():
        if v.is_floating_point():
            assert rel(sd[k], v) < tol, k
        else:
            assert torch.equal(sd[k].cpu(), v), k


def _step(model, opt, x, eps, cfg):
    opt.zero_grad(set_to_none=True)
    y, mu, logstd = model(x, eps)
    R = fv.ReconLoss()((x, y))
    K = fv.KLDivergenceLoss()((mu, logstd))
    (cfg.w_R * R + cfg.w_K * K).backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    opt.step()
    return y, mu, R, K, grads


def dead_bias(cfg):
    return {s.prefix + ".bias" for s in O.conv_specs(cfg)
            if s.block == "cna" or (s.block == "nac" and ".layers.0.layers.2" in s.prefix)}


def test_toy_training_step_matches_reference_fp32():
    g = load("toy_step.pt")
    cfg = fv.FaceVAEConfig.toy()
    ocfg = O.OracleConfig.toy()
    m = fv.FaceVAE(cfg)
    m.load_state_dict(g["init"])
    m = m.cuda().train().set_compute_dtype(torch.float32)
    opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
    x, eps = g["x"].cuda(), g["eps"].cuda()
    y, mu, R, K, grads = _step(m, opt, x, eps, cfg)
    s1 = g["step1"]
    assert rel(y, s1["y"]) < 1e-4
    assert rel(mu, s1["mu"]) < 1e-4
    assert abs(R.item() - s1["R"].item()) < 1e-4 * s1["R"].item()
    assert abs(K.item() - s1["K"].item()) < 1e-4 * abs(s1["K"].item())
    dead = dead_bias(ocfg)
    for k, gr in s1["grads"].items():
        if k in dead:
            assert (grads[k].cpu() - gr).abs().max() < 1e-4, k
        else:
            assert rel(grads[k], gr) < 1e-3, k
    sd = m.state_dict()
    for k, v in s1["state"].items():
        if not v.is_floating_point():
            assert torch.equal(sd[k].cpu(), v), k
        elif k in dead:
            assert (sd[k].cpu() - v).abs().max() <= 2 * cfg.lr + 1e-6, k
        else:
            assert rel(sd[k], v) < 1e-4, k
    Rs, Ks = [R.item()], [K.item()]
    for _ in range(2):
        y, _, R, K, _ = _step(m, opt, x, eps, cfg)
        Rs.append(R.item())
        Ks.append(K.item())
    torch.cuda.synchronize()
    assert torch.allclose(torch.tensor(Rs, dtype=torch.float64), g["step3"]["R"].double(), rtol=1e-3)
    assert torch.allclose(torch.tensor(Ks, dtype=torch.float64), g["step3"]["K"].double(), rtol=1e-3)
    assert rel(y, g["step3"]["y"]) < 1e-3


@pytest.fixture(scope="module")
def full_oracle():
    """Oracle (CPU fp32) run of two training steps at 256x256, B=2 (the north_star parity case)."""
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = O.OracleConfig()
    sd = O.prepare_state(O.init_state(cfg, 0))
    opt = O.adam_init(sd)
    x = torch.rand(2, 3, 256, 256, generator=torch.Generator().manual_seed(1234))
    eps = torch.randn(2, 256, 64, 64, generator=torch.Generator().manual_seed(1235))
    outs = []
    for _ in range(2):
        o, _ = O.train_step(sd, opt, x, eps, cfg)
        outs.append({k: v.detach() for k, v in o.items()})
    return x, eps, outs


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_full256_step_matches_oracle(full_oracle, dtype):
    x, eps, outs = full_oracle
    g = load("full256.pt")
    torch.manual_seed(0)
    cfg = fv.FaceVAEConfig()
    m = fv.FaceVAE(cfg).cuda().train().set_compute_dtype(dtype)
    opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
    xc, ec = x.cuda(), eps.cuda()
    res = []
    for _ in range(2):
        y, mu, R, K, _ = _step(m, opt, xc, ec, cfg)
        res.append((y.detach().cpu(), R.item(), K.item()))
    torch.cuda.synchronize()
    dev = {
        "image": max(rel(res[i][0], outs[i]["y"]) for i in range(2)),
        "R": max(abs(res[i][1] - outs[i]["R"].item()) / outs[i]["R"].item() for i in range(2)),
        "K": max(abs(res[i][2] - outs[i]["K"].item()) / abs(outs[i]["K"].item()) for i in range(2)),
    }
    print(f"\n[{dtype}] 256x256 B=2 deviation vs oracle over 2 steps: {dev}")
    # the oracle itself matches the reference's fixture (tests/test_oracle_golden.py)
    assert abs(outs[0]["R"].item() - g["R"][0].item()) < 1e-5 * g["R"][0].item()
    if dtype == torch.float32:
        assert dev["image"] < 1e-3 and dev["R"] < 1e-3 and dev["K"] < 1e-3
    else:
        # deterministic kernels: r6 measured image 5.7e-3 / 5.5e-3 (256 / 512), R <= 2.0e-4,
        # K <= 8.5e-5 on every box -- the losses hold the north_star 1e-3 bar in bf16 too
        assert dev["image"] < 1e-2 and dev["R"] < 1e-3 and dev["K"] < 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_full512_step_matches_oracle(dtype):
    """BASELINE config C4 (512x512 high-res VAE): every spatial extent doubles (latent 128x128,
    AFE.in_conv / UpBlock2 at 512x512), so each kernel runs at shapes the 256 case never
    reaches.  One step at B=1 vs the CPU oracle (fp32 mode 1e-3; bf16 image 1e-2, losses 1e-3),
    plus the step-2 losses (after Adam on the GPU vs Adam on the oracle)."""
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ocfg = O.OracleConfig(H=512)
    torch.manual_seed(0)
    cfg = fv.FaceVAEConfig.hires()
    m = fv.FaceVAE(cfg)
    init = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.cuda().train().set_compute_dtype(dtype)
    opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
    x = torch.rand(1, 3, 512, 512, generator=torch.Generator().manual_seed(1234))
    eps = torch.randn(1, 256, 128, 128, generator=torch.Generator().manual_seed(1235))
    sd = O.prepare_state(init)
    ost = O.adam_init(sd)
    outs = []
    for _ in range(2):
        o, _ = O.train_step(sd, ost, x, eps, ocfg)
        outs.append({k: v.detach() for k, v in o.items()})
    xc, ec = x.cuda(), eps.cuda()
    res = []
    for _ in range(2):
        y, mu, R, K, _ = _step(m, opt, xc, ec, cfg)
        res.append((y.detach().cpu(), R.item(), K.item()))
    torch.cuda.synchronize()
    dev = {
        "image": max(rel(res[i][0], outs[i]["y"]) for i in range(2)),
        "R": max(abs(res[i][1] - outs[i]["R"].item()) / outs[i]["R"].item() for i in range(2)),
        "K": max(abs(res[i][2] - outs[i]["K"].item()) / abs(outs[i]["K"].item()) for i in range(2)),
    }
    print(f"\n[{dtype}] 512x512 B=1 deviation vs oracle over 2 steps: {dev}")
    if dtype == torch.float32:
        assert dev["image"] < 1e-3 and dev["R"] < 1e-3 and dev["K"] < 1e-3
    else:
        # deterministic kernels: r6 measured image 5.7e-3 / 5.5e-3 (256 / 512), R <= 2.0e-4,
        # K <= 8.5e-5 on every box -- the losses hold the north_star 1e-3 bar in bf16 too
        assert dev["image"] < 1e-2 and dev["R"] < 1e-3 and dev["K"] < 1e-3


def test_trainer_surface(tmp_path):
    cfg = fv.FaceVAEConfig.toy()
    batch = [(torch.rand(2, 3, 64, 64),) * 4 for _ in range(2)]
    tr = fv.FaceVAETrainer(str(tmp_path / "ckp"), str(tmp_path / "vis"), batch, lr=5e-5, cfg=cfg,
                           log_file_name=str(tmp_path / "log.txt"))
    tr.step()
    assert os.path.exists(tmp_path / "ckp" / "00000000-checkpoint.pth.tar")
    txt = open(tmp_path / "log.txt").read()
    assert txt.startswith("G00000000) R - ") and "; K - " in txt
    tr2 = fv.FaceVAETrainer(str(tmp_path / "ckp"), None, batch, lr=5e-5, cfg=cfg,
                            log_file_name=str(tmp_path / "log2.txt"))
    tr2.load_cpk(0)
    assert tr2.epoch == 1
    for (k, a), (_, b) in zip(tr.model.state_dict().items(), tr2.model.state_dict().items()):
        assert torch.equal(a.cpu(), b.cpu()), k
