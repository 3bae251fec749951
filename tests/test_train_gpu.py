"""The reference launch path end to end (train.py:10-54): `python train.py` spawns one process
per rank (mp.spawn), each seeds (init_seeds), rendezvouses (init_dist or a bare torch process
group as the reference's own init_dist creates), reads its DistributedSampler shard of the
dataset, and runs FaceVAETrainer.step() per epoch (the Logger surface).  Two ranks share the
one GPU of the box over gloo (RCCL refuses two ranks on one device).  After an epoch every
rank must hold identical parameters (gradients averaged, rank 0's init broadcast), the master
writes the checkpoint and the loss log."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("init", ["ours", "torch"])
def test_train_py_two_ranks(tmp_path, init):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29500 + (os.getpid() % 1000) + (init == "torch")))
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "--gpu_ids", "[0,1]", "--backend", "gloo", "--config", "toy",
           "--synthetic", "8", "--batch_size", "2", "--num_epochs", "1", "--num_workers", "0", "--init", init,
           "--ckp_dir", str(tmp_path / "ckp"), "--vis_dir", str(tmp_path / "vis"),
           "--log_file", str(tmp_path / "logs" / "log.txt"), "--dump_dir", str(tmp_path / "dump")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    s0 = torch.load(tmp_path / "dump" / "rank0.pt", weights_only=True)
    s1 = torch.load(tmp_path / "dump" / "rank1.pt", weights_only=True)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    # 8 samples / 2 ranks / batch 2 = 2 steps: the BN counter advanced twice on every rank
    nbt = [v for k, v in s0.items() if k.endswith("num_batches_tracked")]
    assert nbt and all(int(v) == 2 for v in nbt)
    assert os.path.exists(tmp_path / "ckpadd" / "00000000-checkpoint.pth.tar")
    # train.py:49: the log goes to <dir of --log_file> + ext + ".txt"
    log = open(str(tmp_path / "logs") + "add.txt").read()
    assert log.startswith("G00000000) R - ")


def test_train_py_single_gpu_graph(tmp_path):
    """train.py on one GPU with --graph true: the first batch captures the step, the rest replay
    it; the epoch completes, the checkpoint and the loss log are written."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + (os.getpid() % 1000)))
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "--gpu_ids", "[0]", "--backend", "gloo", "--config", "toy",
           "--synthetic", "8", "--batch_size", "2", "--num_epochs", "1", "--num_workers", "0", "--graph", "true",
           "--ckp_dir", str(tmp_path / "ckp"), "--vis_dir", str(tmp_path / "vis"),
           "--log_file", str(tmp_path / "logs" / "log.txt"), "--dump_dir", str(tmp_path / "dump")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    s0 = torch.load(tmp_path / "dump" / "rank0.pt", weights_only=True)
    nbt = [v for k, v in s0.items() if k.endswith("num_batches_tracked")]
    assert nbt and all(int(v) == 4 for v in nbt)      # 8 samples / batch 2: 4 steps, 3 of them replayed
    log = open(str(tmp_path / "logs") + "add.txt").read()
    assert log.startswith("G00000000) R - ")
