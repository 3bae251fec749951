#!/bin/bash
# A/B of the v2 forward k loop (FV_CONV_DBG=8: reference loop) after the parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
rm -f gpurun_out/fwdab.log
for d in 8 0 ${EXTRA_DBG:-}; do
  echo "== FV_CONV_DBG=$d" >> gpurun_out/fwdab.log
  FV_CONV_DBG=$d timeout -k 10 200 python tools/convbench.py --only fwd,dgrad --iters 10 >> gpurun_out/fwdab.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
python tools/benchline.py < gpurun_out/bench.log
