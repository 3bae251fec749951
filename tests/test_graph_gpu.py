"""HIP-graph step replay (graph.StepGraph) against the eager step, on the same weights and
inputs.

Tolerances: the graph replays the same kernels on the same operands, so images, losses and
parameters agree to fp32 rounding of the Adam coefficients (device fp64 pow against the host's:
1e-6 relative).  The graph step is also checked against the reference fixture (toy_step.pt,
step 3) at the north_star bar of 1e-3.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402
from facevae_amd import ops  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _setup(dtype, init=None, H=None):
    cfg = fv.FaceVAEConfig.toy() if H is None else fv.FaceVAEConfig(H=H)
    torch.manual_seed(0)
    m = fv.FaceVAE(cfg)
    if init is not None:
        m.load_state_dict(init)
    m = m.cuda().train().set_compute_dtype(dtype)
    opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
    return cfg, m, opt


def _step_fn(m, opt, x, eps, cfg):
    rec, kl = fv.ReconLoss(), fv.KLDivergenceLoss()

    def step():
        opt.zero_grad(set_to_none=True)
        y, mu, logstd = m(x, eps)
        R = rec((x, y))
        K = kl((mu, logstd))
        (cfg.w_R * R + cfg.w_K * K).backward()
        opt.step()
        return y.detach(), R.detach(), K.detach()
    return step


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_graph_replay_matches_eager(dtype):
    g = torch.load(os.path.join(GOLD, "toy_step.pt"), weights_only=True)
    x, eps = g["x"].cuda(), g["eps"].cuda()
    cfg, ma, oa = _setup(dtype, g["init"])
    sa = _step_fn(ma, oa, x, eps, cfg)
    for _ in range(5):
        ya, Ra, Ka = sa()
    torch.cuda.synchronize()

    cfg, mb, ob = _setup(dtype, g["init"])
    sb = _step_fn(mb, ob, x, eps, cfg)
    graph = fv.StepGraph(sb, [ob], warmup=2).capture()
    for _ in range(3):
        yb, Rb, Kb = graph.replay()
    torch.cuda.synchronize()
    assert rel(yb, ya) < 1e-6 and abs(Rb.item() - Ra.item()) <= 1e-6 * abs(Ra.item())
    assert abs(Kb.item() - Ka.item()) <= 1e-6 * abs(Ka.item())
    pa, pb = dict(ma.named_parameters()), dict(mb.named_parameters())
    for k in pa:
        assert rel(pb[k], pa[k]) < 1e-6, k
    ba, bb = dict(ma.named_buffers()), dict(mb.named_buffers())
    for k in ba:
        if ba[k].is_floating_point():
            assert rel(bb[k], ba[k]) < 1e-6, k
        else:
            assert torch.equal(bb[k], ba[k]), k
    # the host step count follows the replays (optimizer checkpoints interchange)
    assert all(int(ob.state[p]["step"].item()) == 5 for p in mb.parameters())
    if dtype == torch.float32:
        # 5 steps from the reference init; the fixture holds steps 1-3 (rtol 1e-3 after 3)
        cfg, mc, oc = _setup(dtype, g["init"])
        sc = _step_fn(mc, oc, x, eps, cfg)
        gc = fv.StepGraph(sc, [oc], warmup=1).capture()
        for _ in range(2):
            yc, Rc, Kc = gc.replay()
        torch.cuda.synchronize()
        assert rel(yc, g["step3"]["y"]) < 1e-3
        assert abs(Rc.item() - g["step3"]["R"][-1].item()) < 1e-3 * g["step3"]["R"][-1].item()


def test_graph_replay_reads_refreshed_inputs():
    """Static inputs refreshed in place between replays drive the captured step."""
    cfg, m, opt = _setup(torch.bfloat16)
    x = torch.rand(2, 3, 64, 64, device="cuda")
    eps = torch.randn(2, cfg.latent, cfg.latent_hw, cfg.latent_hw, device="cuda")
    graph = fv.StepGraph(_step_fn(m, opt, x, eps, cfg), [opt], warmup=1).capture()
    y1 = graph.replay()[0].clone()
    x.copy_(torch.rand_like(x))
    y2 = graph.replay()[0].clone()
    torch.cuda.synchronize()
    assert rel(y2, y1) > 1e-3


def test_graph_replay_256_bench_shape():
    """The bench's configuration (256x256, bf16) replays: finite losses, parameters moving."""
    cfg, m, opt = _setup(torch.bfloat16, H=256)
    B = 4
    x = torch.rand(B, 3, 256, 256, device="cuda")
    eps = torch.randn(B, cfg.latent, cfg.latent_hw, cfg.latent_hw, device="cuda")
    graph = fv.StepGraph(_step_fn(m, opt, x, eps, cfg), [opt], warmup=1).capture()
    w0 = m.afe.in_conv.conv.weight.detach().clone() if hasattr(m, "afe") else next(m.parameters()).detach().clone()
    for _ in range(2):
        y, R, K = graph.replay()
    torch.cuda.synchronize()
    assert torch.isfinite(R).item() and torch.isfinite(K).item()
    w1 = m.afe.in_conv.conv.weight.detach() if hasattr(m, "afe") else next(m.parameters()).detach()
    assert not torch.equal(w0, w1)


def test_trainer_graph_mode_matches_eager():
    """FaceVAETrainer(graph=True): the first batch captures, later batches of that shape replay,
    a batch of another shape runs eagerly -- and replays resume after it (batch sizes
    2, 2, 1, 2, 2: replay -> eager -> replay).  After EVERY step the losses, all parameters and
    the Adam step counts equal the eager trainer's (the eager step in between must see the
    device step counter the replays advanced, and re-prepare the weights the graph shape had
    prepared)."""
    g = torch.load(os.path.join(GOLD, "toy_step.pt"), weights_only=True)
    cfg = fv.FaceVAEConfig.toy()
    sizes = [2, 2, 1, 2, 2]
    trs = []
    for graph in (False, True):
        torch.manual_seed(0)
        tr = fv.FaceVAETrainer(None, None, [], cfg.lr, cfg=cfg, compute_dtype=torch.float32, graph=graph)
        tr.model.load_state_dict(g["init"])
        trs.append(tr)
    gen = torch.Generator().manual_seed(7)
    for i, B in enumerate(sizes):
        x = torch.rand(B, 3, 64, 64, generator=gen).cuda()
        eps = torch.randn(B, cfg.latent, cfg.latent_hw, cfg.latent_hw, generator=gen).cuda()
        outs = [tr.train_step(x, eps) for tr in trs]
        torch.cuda.synchronize()
        (ra, ka), (rb, kb) = [(o["R"].item(), o["K"].item()) for o in outs]
        assert abs(ra - rb) <= 1e-6 * abs(ra) and abs(ka - kb) <= 1e-6 * abs(ka), (i, ra, rb, ka, kb)
        pa, pb = dict(trs[0].model.named_parameters()), dict(trs[1].model.named_parameters())
        for k in pa:
            assert rel(pb[k], pa[k]) < 1e-6, (i, k)
        for name in trs[0].g_optimizers:
            oa, ob = trs[0].g_optimizers[name], trs[1].g_optimizers[name]
            sa = [int(oa.state[p]["step"].item()) for p in oa.param_groups[0]["params"]]
            sb = [int(ob.state[p]["step"].item()) for p in ob.param_groups[0]["params"]]
            assert sa == sb == [i + 1] * len(sa), (i, name, sa[:3], sb[:3])
    assert trs[1]._sg is not None            # the graph of the first shape survived the eager step


@pytest.mark.parametrize("graph", [False, True])
def test_trainer_loss_weights_seed_backward(graph):
    """FaceVAETrainer seeds the backward of R and K with their weights (no ones-fill / add /
    scalar multiplies in the step): with the reference's commented weights (w_R = 10, w_K = 0.2,
    trainer.py:250-251) three steps give the parameters and losses of the plain
    (w_R R + w_K K).backward() step on the same model -- bit-identical eager, within the
    graph-vs-eager Adam bar when graph-replayed."""
    import dataclasses
    g = torch.load(os.path.join(GOLD, "toy_step.pt"), weights_only=True)
    cfg = dataclasses.replace(fv.FaceVAEConfig.toy(), w_R=10.0, w_K=0.2)
    torch.manual_seed(0)
    tr = fv.FaceVAETrainer(None, None, [], cfg.lr, cfg=cfg, compute_dtype=torch.float32, graph=graph)
    tr.model.load_state_dict(g["init"])
    torch.manual_seed(0)
    m = fv.FaceVAE(cfg).cuda().set_compute_dtype(torch.float32)
    m.load_state_dict(g["init"])
    opts = [fv.Adam(mm.parameters(), lr=cfg.lr, betas=cfg.betas) for mm in (m.afe, m.generator)]
    rec, kl = fv.ReconLoss(), fv.KLDivergenceLoss()
    gen = torch.Generator().manual_seed(3)
    for i in range(3):
        x = torch.rand(2, 3, 64, 64, generator=gen).cuda()
        eps = torch.randn(2, cfg.latent, cfg.latent_hw, cfg.latent_hw, generator=gen).cuda()
        out = tr.train_step(x, eps)
        for o in opts:
            o.zero_grad(set_to_none=True)
        y, mu, ls = m(x, eps)
        R, K = rec((x, y)), kl((mu, ls))
        (cfg.w_R * R + cfg.w_K * K).backward()
        for o in opts:
            o.step()
        torch.cuda.synchronize()
        # eager: bit-identical; graph: the replayed Adam's device-side bias correction differs
        # from the eager one in the last bits (test_trainer_graph_mode_matches_eager's bar)
        tol = 1e-6 if graph else 0.0
        for a, b in ((out["R"].item(), (cfg.w_R * R).item()), (out["K"].item(), (cfg.w_K * K).item())):
            assert abs(a - b) <= tol * abs(b), (i, a, b)
        pa = dict(tr.model.named_parameters())
        for k, p in m.named_parameters():
            assert (rel(pa[k], p) < 1e-6) if graph else torch.equal(pa[k], p), (i, k)


def test_sn_bwd_batch_bit_identical(monkeypatch):
    """Spectral-norm backward terms batched at the end of backward (ops._SN_BATCH) against the
    per-conv launches: the same partial sums in the same order, bit-identical parameters."""
    g = torch.load(os.path.join(GOLD, "toy_step.pt"), weights_only=True)
    x, eps = g["x"].cuda(), g["eps"].cuda()
    out = []
    for batch in (False, True):
        monkeypatch.setattr(ops, "_SN_BATCH", batch)
        cfg, m, opt = _setup(torch.float32, g["init"])
        s = _step_fn(m, opt, x, eps, cfg)
        for _ in range(2):
            s()
        torch.cuda.synchronize()
        out.append({k: p.detach().clone() for k, p in m.named_parameters()})
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k


def test_segmented_capture_that_raises_leaves_capture_mode():
    """when the captured step raises inside a segmented (world > 1) capture, the open
    segment is ended, so the capture stream is usable afterwards and the error surfaces.  A
    stand-in communicator with world_size 2 selects the segmented path; the step fails before
    any collective."""
    from facevae_amd import distributed as D

    class _FakeComm:
        world_size, rank = 2, 0

    x = torch.randn(1 << 16, device="cuda")

    def bad_step():
        y = x * 2.0 + 1.0
        if y.numel() > 0:
            raise ValueError("step failed inside the capture")
        return y

    prev = (D._COMM, D._SYNCBN)
    D.install(_FakeComm(), syncbn=False)
    try:
        calls = {"n": 0}

        def step():                          # the eager warm-up call succeeds, the captured one raises
            calls["n"] += 1
            return x * 3.0 if calls["n"] == 1 else bad_step()
        with pytest.raises(ValueError, match="inside the capture"):
            fv.StepGraph(step, [], warmup=1).capture()
    finally:
        D.install(*prev)
    assert not torch.cuda.is_current_stream_capturing()
    z = (x + 1.0).sum()                      # ordinary GPU work and a new capture still run
    torch.cuda.synchronize()
    assert torch.isfinite(z).item()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        w = x * 5.0
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(w, x * 5.0)
