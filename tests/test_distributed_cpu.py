"""Data-parallel plumbing on CPU: world_size 2 over gloo (torch.distributed), through the same
DataParallel / TorchComm code the GPU path drives over RCCL (distributed.py).

Checks the DDP contract the reference relies on (logger.py:55,58 -> torch DDP): the initial
parameter broadcast from rank 0 (collective C2), gradient averaging across
ranks in buckets (C4) so that each rank ends with the gradient of the global-batch mean
loss, and the buffer sync (C3).  The model here is plain torch (CPU); the bucketing,
hooks, flat buffers and averaging are the product code.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(6, 5)
        self.b = torch.nn.Linear(5, 3)
        self.register_buffer("running", torch.zeros(3))

    def forward(self, x):
        return self.b(torch.tanh(self.a(x)))


def _worker(rank, world, port, bucket_mb, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import fvamd  # noqa: F401
        from facevae_amd import distributed as D
        torch.manual_seed(100 + rank)            # deliberately different init per rank
        net = _Net()
        net.running.fill_(float(rank + 1))
        comm = D.TorchComm()
        D.install(comm, syncbn=True)
        dp = D.DataParallel(net, comm, bucket_cap_mb=bucket_mb)
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
        q.put((rank, flat, grads, len(dp.buckets), D.syncbn_comm() is comm))
    finally:
        dist.destroy_process_group()


def _run(world, bucket_mb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


@pytest.mark.parametrize("bucket_mb", [25.0, 1e-6])
def test_dataparallel_gloo_world2(bucket_mb):
    out = _run(2, bucket_mb)
    (_, f0, g0, nb0, sb0), (_, f1, g1, nb1, sb1) = out
    assert torch.equal(f0, f1), "rank-0 broadcast of params/buffers"
    assert sb0 and sb1, "SyncBN communicator installed"
    if bucket_mb < 1:
        assert nb0 == 4, "tiny cap: one bucket per parameter"
    else:
        assert nb0 == 1
    assert torch.allclose(g0, g1, atol=0, rtol=0), "identical averaged gradients on every rank"
    # reference: the same model on the global batch (mean loss) in one process
    torch.manual_seed(100)
    ref = _Net()
    g = torch.Generator().manual_seed(7)
    xs = torch.randn(4, 6, generator=g)
    ys = torch.randn(4, 3, generator=g)
    loss = ((ref(xs) - ys) ** 2).mean()
    loss.backward()
    gr = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    assert torch.allclose(g0, gr, rtol=1e-5, atol=1e-6)
