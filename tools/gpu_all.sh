#!/bin/bash
# tests + bench + (optional) PMC passes in one box session
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
if [ -n "$PMC" ]; then bash tools/gpu_pmc.sh || exit 1; fi
if [ -n "$CONVBENCH_ARGS" ]; then timeout -k 10 300 python tools/convbench.py $CONVBENCH_ARGS > gpurun_out/convbench.log 2>&1 || exit 1; fi
