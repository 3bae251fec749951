"""The RCCL communicator of the data-parallel path (fv_comm_*, comm.cpp; RcclComm in
distributed.py) on the real GPU at world_size 1 -- the only RCCL shape a one-GPU box admits
(RCCL refuses two ranks on one device; the multi-rank SyncBN / gradient-averaging logic is
covered by tests/test_distributed_gpu.py over gloo and tests/test_distributed_cpu.py).
Checks unique-id exchange, communicator init, all-reduce (sum / avg) in fp32 / bf16 / fp64,
broadcast, all-gather and destroy, stream-ordered on a side stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import fvamd  # noqa: E402,F401
import facevae_amd as fv  # noqa: E402


def test_rccl_world1_collectives():
    D = fv.distributed
    torch.cuda.set_device(0)
    uid = D.RcclComm.unique_id()
    assert len(uid) == 128 and any(uid)
    comm = D.RcclComm(0, 1, 0, uid)
    try:
        # collectives run on the communicator's own stream, fenced against the caller's
        # stream: a kernel queued just before must be seen, the caller sees the result after
        # wait_back (SyncBN) or after fence() (gradient buckets)
        for dt in (torch.float32, torch.bfloat16, torch.float64):
            t = torch.zeros(1 << 20, device="cuda").to(dt)
            ref = torch.randn(1 << 20, device="cuda").to(dt)
            t.copy_(ref)                                      # queued on the caller's stream
            comm.allreduce_(t, op="sum")                      # wait_back=True
            comm.allreduce_(t, op="avg", wait_back=False)
            comm.fence()
            assert torch.equal(t, ref), dt                   # one rank: sum and avg are identities
        b = torch.arange(1000, dtype=torch.float32, device="cuda")
        comm.broadcast_(b, 0)
        assert torch.equal(b.cpu(), torch.arange(1000, dtype=torch.float32))
        g = torch.empty(1000, dtype=torch.float32, device="cuda")
        fv._lib.call("fv_comm_allgather", comm._h, b.data_ptr(), g.data_ptr(), 1000, fv._lib.dtype_code(b.dtype),
                     fv._lib.stream())
        torch.cuda.synchronize()
        assert torch.equal(g, b)
    finally:
        comm.destroy()


def test_rccl_failure_detection_world1():
    """the async-error query of a healthy communicator returns success
    (ncclSuccess) before and after collectives, ncclCommCount sees the one rank, a watchdog
    around the communicator tracks the collectives to completion without firing, and abort
    frees it (later collectives raise instead of touching a dead handle)."""
    D = fv.distributed
    torch.cuda.set_device(0)
    comm = D.RcclComm(0, 1, 0, D.RcclComm.unique_id())
    assert comm.watchdog is None                       # world 1: nothing can hang
    assert comm.async_error() == 0 and comm.count() == 1
    fired = []
    comm.watchdog = D.CommWatchdog(0, comm.async_error, lambda: fired.append("abort"), timeout_s=60, poll_s=0.05,
                                   exit_fn=lambda c: fired.append(c))
    t = torch.randn(1 << 20, device="cuda")
    for _ in range(4):
        comm.allreduce_(t, op="sum", wait_back=False)
    comm.fence()
    torch.cuda.synchronize()
    assert comm.watchdog.check() is None and comm.watchdog.pending() == 0
    assert comm.async_error() == 0 and fired == []
    comm.watchdog.stop()
    comm.watchdog = None
    comm.abort()
    with pytest.raises(RuntimeError):
        comm.allreduce_(t, op="sum")
    comm.destroy()                                      # no-op after abort


def test_dataparallel_over_rccl_world1_is_transparent():
    """DataParallel around the toy model with a world-1 RCCL communicator: no hooks, no
    broadcast, the step equals the bare model's step bit for bit."""
    D = fv.distributed
    cfg = fv.FaceVAEConfig.toy()
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1)).cuda()
    eps = torch.randn(2, 16, 32, 32, generator=torch.Generator().manual_seed(2)).cuda()
    outs = []
    for wrap in (False, True):
        torch.manual_seed(0)
        m = fv.FaceVAE(cfg).cuda().train()
        comm = D.RcclComm(0, 1, 0, D.RcclComm.unique_id()) if wrap else None
        net = D.DataParallel(m, comm) if wrap else m
        y, mu, logstd = net(x, eps)
        (fv.ReconLoss()((x, y)) + fv.KLDivergenceLoss()((mu, logstd))).backward()
        torch.cuda.synchronize()
        outs.append((y.detach().clone(), [p.grad.clone() for p in m.parameters()]))
        if comm is not None:
            comm.destroy()
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert torch.equal(a, b)
