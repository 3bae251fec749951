"""Data-parallel step of the REAL HIP model with SyncBN semantics (SURVEY.md §8e "Parity at
N GPUs"): world_size 2, both ranks on cuda:0 of the one-GPU box, collectives over gloo
(TorchComm: RCCL refuses two ranks on one device; the DataParallel buckets / hooks and the
SyncBN stats + backward-sum all-reduces are the same product code the RCCL communicator
drives).  Each rank steps on its half of a global batch of 4; with SyncBN and averaged
gradients this must equal the single-process global-batch step of the CPU oracle (fp32
mode, 1e-3 relative, the north_star tolerance).
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


def _inputs():
    B = WORLD * PER_RANK
    x = torch.rand(B, 3, 64, 64, generator=torch.Generator().manual_seed(1234))
    eps = torch.randn(B, 16, 32, 32, generator=torch.Generator().manual_seed(1235))
    return x, eps


def _worker(rank, port, q):
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
        cfg = fv.FaceVAEConfig.toy()
        torch.manual_seed(10 + rank)                 # different init per rank: rank 0's is broadcast
        m = fv.FaceVAE(cfg).cuda().train().set_compute_dtype(torch.float32)
        dp = D.DataParallel(m, comm)
        opt = fv.Adam(m.parameters(), lr=cfg.lr, betas=cfg.betas)
        x, eps = _inputs()
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


def test_dataparallel_syncbn_two_ranks_match_global_batch_oracle():
    from oracle import facevae_cpu as O          # checker only
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
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
    (_, R0, K0, y0, init0, g0, a0), (_, R1, K1, y1, init1, g1, a1) = out
    # C2: rank 0's parameters / buffers broadcast before the step
    for k in init0:
        assert torch.equal(init0[k], init1[k]), k

    x, eps = _inputs()
    ocfg = O.OracleConfig.toy()
    sd = O.prepare_state(init0)
    oo, og = O.train_step(sd, O.adam_init(sd), x, eps, ocfg)

    def rel(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()

    # global-batch losses = mean of the per-rank means (equal shards)
    assert abs((R0 + R1) / 2 - oo["R"].item()) < 1e-3 * oo["R"].item()
    assert abs((K0 + K1) / 2 - oo["K"].item()) < 1e-3 * abs(oo["K"].item())
    assert rel(torch.cat([y0, y1]), oo["y"]) < 1e-3           # SyncBN: global-batch statistics
    dead = {s.prefix + ".bias" for s in O.conv_specs(ocfg)
            if s.block == "cna" or (s.block == "nac" and ".layers.0.layers.2" in s.prefix)}
    for k, g in og.items():
        assert torch.equal(g0[k], g1[k]), k                   # identical averaged gradients
        if k in dead:
            assert (g0[k] - g).abs().max() < 1e-4, k
        else:
            assert rel(g0[k], g) < 1e-3, k
    for k, v in sd.items():
        if v.is_floating_point() and k not in dead:
            assert rel(a0[k], v.detach()) < 1e-4, k
        elif not v.is_floating_point():
            assert torch.equal(a0[k], v), k
