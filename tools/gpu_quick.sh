#!/bin/bash
# Iteration run: GPU parity tests, per-layer conv timings, step bench (no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/convbench.py ${CONVBENCH_ARGS:-} > gpurun_out/convbench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
python tools/benchline.py < gpurun_out/bench.log
