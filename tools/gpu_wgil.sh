#!/bin/bash
# wgrad interleave bring-up: kernel tests, convbench A/B (FV_WG_IL), full-step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_layers_gpu.py > gpurun_out/wgil_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wgil_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/wgil_tests.log | head; exit 1; }
: > gpurun_out/wgil_ab.log
for i in 1 2; do
  for v in FV_WG_IL=0 FV_WG_IL=1; do
    echo "== $v" >> gpurun_out/wgil_ab.log
    env $v timeout -k 10 200 python tools/convbench.py --only wgrad >> gpurun_out/wgil_ab.log 2>&1 || exit 1
  done
done
AB_KNOB=FV_WG_IL=0 AB_REPS=3 bash tools/gpu_ab_bench.sh
