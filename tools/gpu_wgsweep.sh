#!/bin/bash
# wgrad tile-config sweep (FV_WG2_CFG) after the parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
rm -f gpurun_out/wgsweep.log
for c in ${CFGS:--1 6 7 8 9 10}; do
  echo "== FV_WG2_CFG=$c" >> gpurun_out/wgsweep.log
  FV_WG2_CFG=$c timeout -k 10 200 python tools/convbench.py --only wgrad --iters 10 >> gpurun_out/wgsweep.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
python tools/benchline.py < gpurun_out/bench.log
