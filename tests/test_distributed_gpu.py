"""Data-parallel step of the REAL HIP model with SyncBN semantics (SURVEY.md §8e "Parity at
N GPUs"): world_size 2, both ranks on cuda:0 of the one-GPU box, collectives over gloo
(TorchComm: RCCL refuses two ranks on one device; the DataParallel buckets / hooks and the
SyncBN stats + backward-sum all-reduces are the same product code the RCCL communicator
drives).  Each rank steps on its half of a global batch of 4; with SyncBN and averaged
gradients this must equal the single-process global-batch step of the CPU oracle (fp32
mode, 1e-3 relative, the north_star tolerance).

The second test runs the REAL 256x256 model in bf16 (the benchmarked kernels: DMA-fed convs,
their BN record layouts and store-pass modes, the quad-pooled DownBlock BN backward) at 2 images
per rank, so the SyncBN sequence partials -> all-reduce -> finalize runs through the timed
kernels, and checks it against the single-process bf16 step at the global batch of 4 on the
same weights and inputs (plus the fp32 oracle at bf16 tolerance).
"""
import io
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2
PER_RANK = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(H=64, latent=16, hw=32, world=WORLD):
    B = world * PER_RANK
    x = torch.rand(B, 3, H, H, generator=torch.Generator().manual_seed(1234))
    eps = torch.randn(B, latent, hw, hw, generator=torch.Generator().manual_seed(1235))
    return x, eps


def _cfg(fv, big):
    return fv.FaceVAEConfig(H=256) if big else fv.FaceVAEConfig.toy()


def _worker(rank, port, q, big=False, world=WORLD, dtype_name=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import fvamd  # noqa: F401
        import facevae_amd as fv
        D = fv.distributed
        torch.cuda.set_device(0)
        comm = D.TorchComm()
        D.install(comm, syncbn=True)
        cfg = _cfg(fv, big)
        torch.manual_seed(10 + rank)                 # different init per rank: rank 0's is broadcast
        mode = getattr(torch, dtype_name) if dtype_name else (torch.bfloat16 if big else torch.float32)
        m = fv.FaceVAE(cfg).cuda().train().set_compute_dtype(mode)
        dp = D.DataParallel(m, comm)
        opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
        x, eps = _inputs(cfg.H, cfg.latent, cfg.latent_hw, world)
        sl = slice(PER_RANK * rank, PER_RANK * (rank + 1))
        xs, es = x[sl].cuda(), eps[sl].cuda()
        init = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        opt.zero_grad(set_to_none=True)
        y, mu, logstd = dp(xs, es)
        R = fv.ReconLoss()((xs, y))
        K = fv.KLDivergenceLoss()((mu, logstd))
        (cfg.w_R * R + cfg.w_K * K).backward()
        grads = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}
        opt.step()
        torch.cuda.synchronize()
        after = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        buf = io.BytesIO()                           # plain bytes: no tensor fd passing
        torch.save((rank, R.item(), K.item(), y.detach().cpu(), init, grads, after), buf)
        q.put(buf.getvalue())
    except Exception as e:                           # surface the failure in the parent
        buf = io.BytesIO()
        torch.save((rank, repr(e), None, None, None, None, None), buf)
        q.put(buf.getvalue())
        raise
    finally:
        dist.destroy_process_group()


def _run_ranks(big, world=WORLD, dtype_name=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, q, big, world, dtype_name)) for r in range(world)]
    for p in ps:
        p.start()
    out = [torch.load(io.BytesIO(q.get(timeout=240)), weights_only=True) for _ in ps]
    out = sorted(out, key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for r in out:
        assert r[2] is not None, f"rank {r[0]} failed: {r[1]}"
    for p in ps:
        assert p.exitcode == 0
    return out


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("world", [2, 8])
def test_dataparallel_syncbn_ranks_match_global_batch_oracle(world):
    """world 2 (global batch 4) and world 8 -- SURVEY §8(e): 8 ranks x 2 images vs the CPU
    restatement at B = 16 (8 gloo ranks on the one GPU: the bucket plan, the SyncBN count rows
    and the fp64 record sums over 8 ranks)."""
    from oracle import facevae_cpu as O          # checker only
    out = _run_ranks(False, world)
    (_, R0, K0, y0, init0, g0, a0) = out[0]
    # C2: rank 0's parameters / buffers broadcast before the step
    for r in out[1:]:
        for k in init0:
            assert torch.equal(init0[k], r[4][k]), (r[0], k)

    x, eps = _inputs(world=world)
    ocfg = O.OracleConfig.toy()

    def oracle(dt):
        sd = O.prepare_state(init0)
        sd = {k: (v.detach().to(dt).requires_grad_(v.requires_grad) if v.is_floating_point() else v.clone())
              for k, v in sd.items()}
        oo, og = O.train_step(sd, O.adam_init(sd), x.to(dt), eps.to(dt), ocfg)
        return sd, oo, og

    sd, oo, og = oracle(torch.float32)
    _, oo64, og64 = oracle(torch.float64)

    def rel(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()

    # global-batch losses = mean of the per-rank means (equal shards)
    Rm = sum(r[1] for r in out) / world
    Km = sum(r[2] for r in out) / world
    assert abs(Rm - oo["R"].item()) < 1e-3 * oo["R"].item()
    assert abs(Km - oo["K"].item()) < 1e-3 * abs(oo["K"].item())
    assert rel(torch.cat([r[3] for r in out]), oo["y"]) < 1e-3   # SyncBN: global-batch statistics
    dead = {s.prefix + ".bias" for s in O.conv_specs(ocfg)
            if s.block == "cna" or (s.block == "nac" and ".layers.0.layers.2" in s.prefix)}
    for k, g in og.items():
        for r in out[1:]:
            assert torch.equal(g0[k], r[5][k]), (r[0], k)     # identical averaged gradients
        if k in dead:
            assert (g0[k] - g).abs().max() < 1e-4, k
        else:
            # vs the float64 oracle: 1e-3, or -- at B = 16 the reference's own fp32 arithmetic is
            # already 3e-3 off float64 on the Generator's first layers (BN-backward cancellation;
            # 1e-6 at B = 4) -- twice the fp32 oracle's own deviation
            e_ref = rel(g, og64[k])
            assert rel(g0[k], og64[k]) < max(1e-3, 2 * e_ref + 1e-4), (k, rel(g0[k], og64[k]), e_ref)
    for k, v in sd.items():
        if v.is_floating_point() and k not in dead:
            assert rel(a0[k], v.detach()) < 1e-4, k
            for r in out[1:]:
                assert torch.equal(a0[k], r[6][k]), (r[0], k)   # every rank: the same step
        elif not v.is_floating_point():
            assert torch.equal(a0[k], v), k


@pytest.mark.parametrize("dtype_name", ["bfloat16", "float8_e4m3fn"])
def test_dataparallel_syncbn_256_two_ranks_match_single_process(dtype_name):
    """Real 256x256 model, bf16 kernels, 2 ranks x 2 images with SyncBN vs one process x 4
    images on the same weights and inputs.  Per-pixel conv outputs do not depend on the batch
    split and the BN statistics / backward sums are fp64 records summed over both ranks, so the
    two runs differ only by summation order (BN records, weight-gradient split-K) and the bf16
    roundings such differences flip: the image, losses, BN running statistics and gradients
    must agree far inside the bf16-vs-fp32 deviation (~2e-2 image).

    float8_e4m3fn (BASELINE config C5's combination): the fp8 convs under DataParallel + SyncBN
    + the gradient all-reduce with GLOBAL delayed scaling: a site's first
    call seeds its history with the exact amax all-reduced (MAX) over the ranks, and every step's
    in-flight amax of all sites is all-reduced in one collective and rolled together
    (DataParallel._sync_fp8), so both ranks quantize with the scales of the 4-image single
    process: the same gates as bf16 (summation order only)."""
    import facevae_amd as fv
    from facevae_amd import distributed as D
    from oracle import facevae_cpu as O          # checker only
    fp8 = dtype_name == "float8_e4m3fn"
    (_, R0, K0, y0, init0, g0, a0), (_, R1, K1, y1, init1, g1, a1) = _run_ranks(True, WORLD, dtype_name)
    for k in init0:
        assert torch.equal(init0[k], init1[k]), k
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k                   # identical averaged gradients

    cfg = fv.FaceVAEConfig(H=256)
    x, eps = _inputs(cfg.H, cfg.latent, cfg.latent_hw)
    D.install(None, syncbn=True)
    m = fv.FaceVAE(cfg)
    m.load_state_dict(init0)
    m = m.cuda().train().set_compute_dtype(getattr(torch, dtype_name))
    opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
    opt.zero_grad(set_to_none=True)
    xc, ec = x.cuda(), eps.cuda()
    y, mu, ls = m(xc, ec)
    R = fv.ReconLoss()((xc, y))
    K = fv.KLDivergenceLoss()((mu, ls))
    (cfg.w_R * R + cfg.w_K * K).backward()
    gs = {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}
    opt.step()
    torch.cuda.synchronize()
    st = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}

    ocfg = O.OracleConfig(H=256)
    sd = O.prepare_state(init0)
    oo, og = O.train_step(sd, O.adam_init(sd), x, eps, ocfg)

    ycat = torch.cat([y0, y1])
    dev = {"image_vs_1proc": _rel(ycat, y.cpu()), "R_vs_1proc": abs((R0 + R1) / 2 - R.item()) / R.item(),
           "K_vs_1proc": abs((K0 + K1) / 2 - K.item()) / abs(K.item()),
           "image_vs_oracle": _rel(ycat, oo["y"]), "R_vs_oracle": abs((R0 + R1) / 2 - oo["R"].item()) / oo["R"].item()}
    dead = {s_.prefix + ".bias" for s_ in O.conv_specs(ocfg)
            if s_.block == "cna" or (s_.block == "nac" and ".layers.0.layers.2" in s_.prefix)}
    gdev = {k: _rel(g0[k], gs[k]) for k in gs if k not in dead}
    # the same gradients, single process vs the fp32 oracle: the bf16 / fp8 floor of each key
    gora = {k: _rel(gs[k], og[k]) for k in gs if k not in dead}
    bn = {k: _rel(a0[k], st[k]) for k in st if k.endswith("running_mean") or k.endswith("running_var")}
    gv = sorted(gdev.values())
    go = sorted(gora.values())
    top = sorted(gdev, key=gdev.get)[-4:]
    print(f"\n[2 ranks x 2, 256x256 {dtype_name}, SyncBN] {dev}\n  grads vs 1 process: median {gv[len(gv) // 2]:.2e} "
          f"(1 process vs oracle: median {go[len(go) // 2]:.2e}); "
          + ", ".join(f"{k} {gdev[k]:.2e} (1 process vs oracle {gora[k]:.2e})" for k in top)
          + f"; BN running stats worst {max(bn.values()):.2e}")
    # (both runs take the same kernels: at 2 and 4 images the latent 256-channel convs are on the
    # 128-co tiles of conv.hip halo3_bn, AFE.down2 on its 256-co tile)
    # measured (r3): forward bit-identical (image 0.0, BN running stats 0.0), K 5e-8; gradients
    # median 2.6e-3.  The worst key, generator.mid_conv.bias (8.4e-2 in r3), is a plain sum over
    # 131,072 pixels of the residual-stream gradient, which is the bf16-rounded sum of the skip
    # gradient and six bn1 backward terms whose pixel sums cancel exactly in real arithmetic:
    # the rounding noise of those terms (a random walk over the pixels) is what is left, and it
    # flips between two summation orders of the fp64 BN sums.  Gated at <= 3e-2 for every other
    # gradient, and for such a sum at twice its own single-process-vs-fp32-oracle deviation
    # (the bf16 floor of that key)
    assert dev["image_vs_1proc"] < 1e-5 and dev["R_vs_1proc"] < 1e-5 and dev["K_vs_1proc"] < 1e-5
    assert dev["image_vs_oracle"] < (5e-2 if fp8 else 2e-2) and dev["R_vs_oracle"] < (1e-2 if fp8 else 1e-3)
    assert gv[len(gv) // 2] < 1e-2
    # fp8 (measured r5): forward bit-identical, gradient median 6.2e-3; the keys above 3e-2 are
    # sums whose e4m3 floor is itself 0.2-0.75 (Generator.in_conv's weight: 7.1e-2 against a
    # 0.75 single-process-vs-oracle deviation; the residual-stream biases) -- two summation
    # orders of the fp64 BN sums flip a few e4m3 roundings of dy, gated at twice that floor
    for k, v in gdev.items():
        assert v <= 3e-2 or ((fp8 or residual_sum_bias(k)) and v <= 2 * gora[k]), (k, v, gora[k])
    assert max(bn.values()) < 1e-5


def residual_sum_bias(k):
    """Conv biases whose gradient is the pixel sum of the ResBlock stack's residual-stream
    gradient: Generator.mid_conv (its output is the stack's input) and every ResBlock's second
    conv (its output is added to the stream).  In bf16 that sum is dominated by the rounding
    noise of the cancelling bn1-backward terms (measured r4: the single process is 8-17 % off
    the fp32 oracle on them)."""
    import re
    return k == "generator.mid_conv.bias" or re.fullmatch(r"generator\.res\.\d+\.layers\.1\.layers\.2\.bias", k) is not None


def _eval_worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import fvamd  # noqa: F401
        import facevae_amd as fv
        D = fv.distributed
        torch.cuda.set_device(0)
        comm = D.TorchComm()
        D.install(comm, syncbn=True)
        torch.manual_seed(10)
        m = fv.FaceVAE(fv.FaceVAEConfig.toy()).cuda().set_compute_dtype(torch.float32)
        dp = D.DataParallel(m, comm)
        m.eval()
        x, eps = _inputs()
        sl = slice(PER_RANK * rank, PER_RANK * (rank + 1))
        xs = x[sl].cuda().requires_grad_(True)
        y, _, _ = dp(xs, eps[sl].cuda())
        g = torch.randn(y.shape, generator=torch.Generator().manual_seed(3 + rank)).cuda()
        (y * g).sum().backward()
        torch.cuda.synchronize()
        buf = io.BytesIO()
        torch.save((rank, xs.grad.cpu(), y.detach().cpu(), g.cpu()), buf)
        q.put(buf.getvalue())
    finally:
        dist.destroy_process_group()


def test_dataparallel_eval_mode_backward_is_local():
    """Backprop through the model in eval mode under DataParallel: BN uses the
    running statistics, so each rank's input gradient must equal a single process's eval-mode
    input gradient for the same images (no SyncBN collective, no finalize on a missing record)."""
    import facevae_amd as fv
    from facevae_amd import distributed as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_eval_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in ps:
        p.start()
    out = sorted([torch.load(io.BytesIO(q.get(timeout=240)), weights_only=True) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    D.install(None, syncbn=True)
    torch.manual_seed(10)
    m = fv.FaceVAE(fv.FaceVAEConfig.toy()).cuda().set_compute_dtype(torch.float32).eval()
    x, eps = _inputs()
    for rank, gx, y_r, g in out:
        sl = slice(PER_RANK * rank, PER_RANK * (rank + 1))
        xs = x[sl].cuda().requires_grad_(True)
        y, _, _ = m(xs, eps[sl].cuda())
        (y * g.cuda()).sum().backward()
        assert _rel(y_r, y.detach().cpu()) < 1e-6
        assert _rel(gx, xs.grad.cpu()) < 1e-5


def _graph_worker(rank, port, q, dtype_name):
    """Rank of the segmented-capture test: model A steps once eagerly, is captured as graph
    segments (every SyncBN / bucket collective and the pre-optimizer fence a segment boundary)
    and replayed twice; model B, the same initial weights, takes three eager steps.  Same
    collectives in the same order on both ranks."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import fvamd  # noqa: F401
        import facevae_amd as fv
        D = fv.distributed
        torch.cuda.set_device(0)
        comm = D.TorchComm()
        D.install(comm, syncbn=True)
        dtype = getattr(torch, dtype_name)
        cfg = fv.FaceVAEConfig.toy()
        x, eps = _inputs(cfg.H, cfg.latent, cfg.latent_hw)
        sl = slice(PER_RANK * rank, PER_RANK * (rank + 1))
        xs, es = x[sl].cuda(), eps[sl].cuda()
        runs = {}
        for mode in ("graph", "eager"):
            torch.manual_seed(10 + rank)
            m = fv.FaceVAE(cfg).cuda().train().set_compute_dtype(dtype)
            dp = D.DataParallel(m, comm)
            opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
            losses = []

            def step():
                opt.zero_grad(set_to_none=True)
                y, mu, logstd = dp(xs, es)
                loss = cfg.w_R * fv.ReconLoss()((xs, y)) + cfg.w_K * fv.KLDivergenceLoss()((mu, logstd))
                loss.backward()
                opt.step()
                return loss

            if mode == "graph":
                sg = fv.StepGraph(step, [opt], warmup=1).capture()
                nseg = len(sg.graph.graphs)
                losses.append(sg.warm_out.item())
                for _ in range(2):
                    losses.append(sg.replay().item())
            else:
                nseg = 0
                for _ in range(3):
                    losses.append(step().item())
            torch.cuda.synchronize()
            runs[mode] = (losses, {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}, nseg)
        buf = io.BytesIO()
        torch.save((rank, runs["graph"][0], runs["eager"][0], runs["graph"][1], runs["eager"][1], runs["graph"][2]),
                   buf)
        q.put(buf.getvalue())
    except Exception as e:
        buf = io.BytesIO()
        torch.save((rank, repr(e), None, None, None, None), buf)
        q.put(buf.getvalue())
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dtype_name", ["float32", "bfloat16"])
def test_dataparallel_segmented_graph_matches_eager(dtype_name):
    """the world > 1 step captured as graph segments between its collectives
    (graph.StepGraph) trains exactly as the eager DataParallel + SyncBN step: 3 steps (1 eager
    warm-up + 2 replays) vs 3 eager steps from the same weights, on both ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_graph_worker, args=(r, port, q, dtype_name)) for r in range(WORLD)]
    for p in ps:
        p.start()
    out = sorted([torch.load(io.BytesIO(q.get(timeout=240)), weights_only=True) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for r in out:
        assert r[2] is not None, f"rank {r[0]} failed: {r[1]}"
    for p in ps:
        assert p.exitcode == 0
    for rank, lg, le, sdg, sde, nseg in out:
        # SyncBN forward + backward all-reduces per BN, the bucket all-reduces and the fence
        assert nseg > 10, nseg
        for a, b in zip(lg, le):
            assert abs(a - b) <= 1e-6 * abs(b), (rank, lg, le)
        for k in sde:
            if sde[k].is_floating_point():
                assert _rel(sdg[k], sde[k]) < 1e-6, (rank, k)
            else:
                assert torch.equal(sdg[k], sde[k]), (rank, k)


def _site_words(m):
    """{module name / operand: the 32 site words} of every fp8 delayed-scaling site of m."""
    out = {}
    for name, mod in m.named_modules():
        for which, st in sorted(mod.__dict__.get("_fv_fp8_sites", {}).items()):
            out[f"{name}/{which}"] = st[0].detach().cpu().clone()
    return out


def _fp8_steps_worker(rank, port, q):
    """Rank of the multi-step fp8 test: the real 256x256 model in fp8 under DataParallel +
    SyncBN, two training steps eagerly and then (same initial weights) one eager warm-up step +
    one replay of the segmented graph; returns every site's words after each run and whether
    the process-wide global-scaling switches were off again after the steps."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import fvamd  # noqa: F401
        import facevae_amd as fv
        D = fv.distributed
        torch.cuda.set_device(0)
        comm = D.TorchComm()
        D.install(comm, syncbn=True)
        cfg = fv.FaceVAEConfig(H=256)
        x, eps = _inputs(cfg.H, cfg.latent, cfg.latent_hw)
        sl = slice(PER_RANK * rank, PER_RANK * (rank + 1))
        xs, es = x[sl].cuda(), eps[sl].cuda()
        res = {}
        for mode in ("eager", "graph"):
            torch.manual_seed(10 + rank)
            m = fv.FaceVAE(cfg).cuda().train().set_compute_dtype(torch.float8_e4m3fn)
            dp = D.DataParallel(m, comm)
            init = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
            opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)

            def step():
                opt.zero_grad(set_to_none=True)
                y, mu, logstd = dp(xs, es)
                loss = cfg.w_R * fv.ReconLoss()((xs, y)) + cfg.w_K * fv.KLDivergenceLoss()((mu, logstd))
                loss.backward()
                opt.step()
                return loss

            if mode == "eager":
                losses = [step().item() for _ in range(2)]
            else:
                sg = fv.StepGraph(step, [opt], warmup=1).capture()
                losses = [sg.warm_out.item(), sg.replay().item()]
            torch.cuda.synchronize()
            off = fv.ops.FP8_GLOBAL is None
            res[mode] = (losses, _site_words(m), off, init)
        buf = io.BytesIO()
        torch.save((rank, res), buf)
        q.put(buf.getvalue())
    except Exception as e:
        buf = io.BytesIO()
        torch.save((rank, repr(e)), buf)
        q.put(buf.getvalue())
        raise
    finally:
        dist.destroy_process_group()


def test_dataparallel_fp8_sites_roll_globally_over_steps():
    """under DataParallel every fp8 site's amax history is rolled once per
    step from the all-reduced (MAX) in-flight amax, so after two steps -- eager, and with the
    segmented graph -- both ranks hold bit-identical site words, matching the single process
    on the global batch of 4 (the step-2 amaxes follow parameters that differ from the single
    process only by gradient summation order); the global-scaling switches are off again after
    the step, and a plain fp8 module in the same process rolls its own sites."""
    import facevae_amd as fv
    from facevae_amd import distributed as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fp8_steps_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in ps:
        p.start()
    out = sorted([torch.load(io.BytesIO(q.get(timeout=400)), weights_only=True) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for r in out:
        assert isinstance(r[1], dict), f"rank {r[0]} failed: {r[1]}"
    r0, r1 = out[0][1], out[1][1]
    for mode in ("eager", "graph"):
        l0, s0, off0, init0 = r0[mode]
        l1, s1, off1, _ = r1[mode]
        assert off0 and off1, mode
        assert len(s0) >= 28 and sorted(s0) == sorted(s1), (mode, len(s0))
        for k in s0:
            assert torch.equal(s0[k], s1[k]), (mode, k)
            assert int(s0[k][17]) == 2, (mode, k, s0[k][17])        # one global roll per step
    ge, gg = r0["eager"][1], r0["graph"][1]
    for k in ge:                                                   # graph replay ~ eager step
        a, b = ge[k][:16].view(torch.float32).double(), gg[k][:16].view(torch.float32).double()
        assert ((a - b).abs() <= 1e-3 * b.abs()).all() and ge[k][17] == gg[k][17], k

    # single process, global batch of 4, same initial weights: two eager fp8 steps
    cfg = fv.FaceVAEConfig(H=256)
    x, eps = _inputs(cfg.H, cfg.latent, cfg.latent_hw)
    D.install(None, syncbn=True)
    assert fv.ops.FP8_GLOBAL is None
    m = fv.FaceVAE(cfg)
    m.load_state_dict(r0["eager"][3])
    m = m.cuda().train().set_compute_dtype(torch.float8_e4m3fn)
    opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
    xc, ec = x.cuda(), eps.cuda()
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        y, mu, ls = m(xc, ec)
        (cfg.w_R * fv.ReconLoss()((xc, y)) + cfg.w_K * fv.KLDivergenceLoss()((mu, ls))).backward()
        opt.step()
    torch.cuda.synchronize()
    s1p = _site_words(m)
    assert sorted(s1p) == sorted(ge)
    # the history of a site after 2 steps: slot 0 = step 1's amax (the single process's seeding
    # call rolls the in-flight word before any quantize pass fed it, so its slot 0 is 0: its
    # scale comes from the 15 seeded slots, which hold the same exact amax), slot 1 = step 2's,
    # slots 2..15 = the seed; the scale is the pow2 of their max
    worst = {"seed": 0.0, "step2": 0.0}
    for k in ge:
        assert int(s1p[k][17]) == int(ge[k][17]), k                # this process rolled its own sites
        a = ge[k][:16].view(torch.float32).double()
        b = s1p[k][:16].view(torch.float32).double()
        # a rank's loss is the mean over its 2 images, so its output gradients are 2x the
        # 4-image process's (the averaged weight gradients are equal): the "dy" amaxes are 2x
        if k.endswith("/dy"):
            b = 2 * b
        r = lambda u, v: abs(u - v).item() / max(abs(v).item(), 1e-30)
        worst["seed"] = max(worst["seed"], r(a[2:].max(), b[2:].max()))
        worst["step2"] = max(worst["step2"], r(a[1], b[1]))
        if k.endswith("/x"):
            # the seed: the same forward up to the fp64 summation order of the SyncBN statistics
            assert r(a[2:].max(), b[2:].max()) <= 1e-4, (k, a.tolist(), b.tolist())
    print(f"\n[fp8 sites, 2 ranks x 2 vs 1 process x 4] amax history worst rel: seed {worst['seed']:.2e}, "
          f"step 2 {worst['step2']:.2e}")
    # (the "dy" seeds are backward amaxes two summation orders apart through e4m3-rounded
    # gradients: measured 1.8e-2 at worst; the step-2 amaxes follow parameters one fp8 step
    # apart -- the e4m3 gradient floor, up to 0.2-0.75 on some keys (test above) -- measured
    # 0.12 at worst: gated loosely, the exact checks are the rank-identity and roll-count ones)
    assert worst["seed"] < 5e-2 and worst["step2"] < 0.3
