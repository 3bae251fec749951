#!/bin/bash
# fwd3 bring-up: kernel + layer tests, then convbench A/B of FV_H3_V3 on the halo layers
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_layers_gpu.py > gpurun_out/v3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/v3_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/v3_tests.log | head; exit 1; }
: > gpurun_out/v3_ab.log
for i in 1 2; do
  for v in FV_H3_V3=0 FV_H3_V3=1; do
    echo "== $v" >> gpurun_out/v3_ab.log
    env $v timeout -k 10 200 python tools/convbench.py --layers res,down2,gin --only fwd,dgrad >> gpurun_out/v3_ab.log 2>&1 || exit 1
  done
done
