"""bench.py's own multi-process step in its default mode (graph segments between the collectives,
VERDICT r4 item 6): two ranks launched by torch.distributed.run on the one GPU of the box, the
collectives over gloo (`--comm gloo`: TorchComm; RCCL refuses two ranks on one device), the full
FaceVAE at 64x64, B=2 per rank.  The bench line must come from the segmented-graph path with both
ranks' images counted, and its last loss must equal the eager run's (same seeds, same number of
optimizer steps: the graph path's capture warm-up and untimed replays are steps too, so the eager
run is given the same total)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(graph, steps, warmup):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", str(warmup),
           "--res", "64", "--batch", "2", "--comm", "gloo", "--cpu-seconds", "0", "--graph", str(graph)]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_graph_segments_match_eager():
    steps, warmup = 3, 2
    g = _bench(1, steps, warmup)
    assert g["n_gpus"] == 2 and g["config"]["global_batch"] == 4
    assert g["launch"].startswith("hip graph segments") and g["comm"] == "gloo"
    assert g["value"] > 0 and g["ms_per_step"] > 0
    # graph path: 1 + (warmup - 1) eager steps, 2 untimed replays, `steps` timed replays
    e = _bench(0, steps + 2, warmup)
    assert e["launch"] == "eager"
    assert abs(g["loss_last"] - e["loss_last"]) <= 1e-5 * abs(e["loss_last"]), (g["loss_last"], e["loss_last"])
