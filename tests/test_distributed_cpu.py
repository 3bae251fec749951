"""Data-parallel plumbing on CPU: world_size 2 over gloo (torch.distributed), through the same
DataParallel / TorchComm code the GPU path drives over RCCL (distributed.py).

Checks the DDP contract the reference relies on (logger.py:55,58 -> torch DDP): the initial
parameter broadcast from rank 0 (collective C2), gradient averaging across
ranks in buckets (C4) so that each rank ends with the gradient of the global-batch mean
loss, and the buffer sync (C3).  The model here is plain torch (CPU); the bucketing,
hooks, flat buffers and averaging are the product code.
"""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(6, 5)
        self.b = torch.nn.Linear(5, 3)
        self.register_buffer("running", torch.zeros(3))

    def forward(self, x):
        return self.b(torch.tanh(self.a(x)))


def _worker(rank, world, store_path, bucket_mb, q, grad_dtype=None):
    # file rendezvous: no TCP port to race for (a probed free port can be taken before the
    # ranks bind it when the container is busy)
    dist.init_process_group("gloo", init_method="file://" + store_path, rank=rank, world_size=world)
    try:
        import fvamd  # noqa: F401
        from facevae_amd import distributed as D
        torch.manual_seed(100 + rank)            # deliberately different init per rank
        net = _Net()
        net.running.fill_(float(rank + 1))
        comm = D.TorchComm()
        D.install(comm, syncbn=True)
        dp = D.DataParallel(net, comm, bucket_cap_mb=bucket_mb, first_bucket_mb=min(bucket_mb, 1.0),
                            grad_dtype=grad_dtype)
        # C2: parameters and buffers now equal rank 0's
        flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()] + [net.running])
        g = torch.Generator().manual_seed(7)
        xs = torch.randn(2 * world, 6, generator=g)
        ys = torch.randn(2 * world, 3, generator=g)
        x, y = xs[2 * rank:2 * rank + 2], ys[2 * rank:2 * rank + 2]
        for _ in range(2):                       # two steps: hooks re-arm every forward
            for p in net.parameters():
                p.grad = None
            loss = ((dp(x) - y) ** 2).mean()
            loss.backward()
        grads = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
        q.put((rank, flat, grads, len(dp.buckets), D.syncbn_comm() is comm, list(dp.launch_order)))
    finally:
        dist.destroy_process_group()


def _run(world, bucket_mb, grad_dtype=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = tempfile.NamedTemporaryFile(prefix="fv_gloo_", delete=False)
    store.close()
    os.unlink(store.name)
    ps = [ctx.Process(target=_worker, args=(r, world, store.name, bucket_mb, q, grad_dtype)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


@pytest.mark.parametrize("world,bucket_mb", [(2, 25.0), (2, 1e-6), (8, 25.0), (8, 1e-6)])
def test_dataparallel_gloo(world, bucket_mb):
    """world 2 and world 8 (the 8-GPU node's rank count, on gloo here)."""
    out = _run(world, bucket_mb)
    (_, f0, g0, nb0, sb0, lo0) = out[0]
    for _, f, g_, nb, sb, lo in out:
        assert torch.equal(f0, f), "rank-0 broadcast of params/buffers"
        assert sb, "SyncBN communicator installed"
        assert nb == nb0 and lo == lo0, "one bucket plan and launch order on every rank"
        assert torch.allclose(g0, g_, atol=0, rtol=0), "identical averaged gradients on every rank"
    if bucket_mb < 1:
        assert nb0 == 4, "tiny cap: one bucket per parameter"
        # buckets hold the parameters in reverse registration order and launch in the order
        # their gradients complete (b.bias / b.weight first: the last layer's grads are ready first)
        assert sorted(lo0) == [0, 1, 2, 3] and set(lo0[:2]) == {0, 1}
    else:
        assert nb0 == 1 and lo0 == [0]
    # reference: the same model on the global batch (mean loss) in one process
    torch.manual_seed(100)
    ref = _Net()
    g = torch.Generator().manual_seed(7)
    xs = torch.randn(2 * world, 6, generator=g)
    ys = torch.randn(2 * world, 3, generator=g)
    loss = ((ref(xs) - ys) ** 2).mean()
    loss.backward()
    gr = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    assert torch.allclose(g0, gr, rtol=1e-5, atol=1e-6)


def test_dataparallel_bf16_grad_compression_world2():
    """grad_dtype=bf16: gradients averaged in a bf16 flat buffer, written back into fp32 .grad
    (the parameter dtype contract holds); equal on both ranks, within bf16 rounding of the
    fp32 global-batch gradient."""
    out = _run(2, 25.0, torch.bfloat16)
    (_, f0, g0, *_), (_, f1, g1, *_) = out
    assert g0.dtype == torch.float32 and torch.equal(g0, g1)
    torch.manual_seed(100)
    ref = _Net()
    g = torch.Generator().manual_seed(7)
    xs = torch.randn(4, 6, generator=g)
    ys = torch.randn(4, 3, generator=g)
    ((ref(xs) - ys) ** 2).mean().backward()
    gr = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    assert ((g0 - gr).norm() / gr.norm()).item() < 1e-2


def test_bucket_plan_faceva_sizes():
    """DDP bucketing of the real FaceVAE parameter set (8,633,091 fp32 params, 34.5 MB):
    a <= 1 MB first bucket holding the last layers (Generator.out_conv ...), then <= 25 MB
    buckets, every parameter exactly once, reverse registration order."""
    import fvamd  # noqa: F401
    from facevae_amd import FaceVAE, FaceVAEConfig
    from facevae_amd.distributed import plan_buckets
    m = FaceVAE(FaceVAEConfig())
    params = [p for p in m.parameters()]
    assert sum(p.numel() for p in params) == 8633091
    bs = plan_buckets(params, 25.0, 1.0)
    sizes = [sum(p.numel() * 4 for p in b) for b in bs]
    assert sizes[0] <= 1 << 20 and all(s <= 25 << 20 for s in sizes[1:])
    assert len(bs) == 3
    flat = [p for b in bs for p in b]
    assert [id(p) for p in flat] == [id(p) for p in reversed(params)]
    assert bs[0][0] is m.generator.out_conv.bias


def test_bn_backward_collective_decision():
    """under a communicator, an eval-mode BN (running statistics: count 0, no
    all-reduced record) takes the local backward -- no all-reduce, k = 0 -- as in a single
    process; training-mode BN keeps the SyncBN path."""
    import fvamd  # noqa: F401
    from facevae_amd import ops

    class _R:
        def __init__(self, count, stats):
            self.count, self.stats = count, stats

    comm = object()
    assert ops.bn_backward_is_local(_R(0, None), None)
    assert ops.bn_backward_is_local(_R(0, None), comm)                  # eval mode under DP
    assert not ops.bn_backward_is_local(_R(None, torch.zeros(3)), comm)  # SyncBN training
    assert ops.bn_backward_is_local(_R(128, None), None)                # single-process training
