#!/bin/bash
# iteration: selected GPU tests, then convbench of selected layers (A/B via env), then bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${TESTS:-tests/test_kernels_gpu.py tests/test_layers_gpu.py} > gpurun_out/pytest_iter.log 2>&1 || { echo "pytest failed"; grep -E "Error|FAIL|assert" gpurun_out/pytest_iter.log | head -20; tail -5 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
timeout -k 10 300 python tools/convbench.py --layers ${LAYERS:-down1} --only ${ONLY:-wgrad} > gpurun_out/cb_a.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/cb_a.log
if [ -n "$AB_ENV" ]; then env $AB_ENV timeout -k 10 300 python tools/convbench.py --layers ${LAYERS:-down1} --only ${ONLY:-wgrad} > gpurun_out/cb_b.log 2>&1 || exit 1; echo "[$AB_ENV]"; grep -v amdgpu.ids gpurun_out/cb_b.log; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
python tools/benchline.py < gpurun_out/bench.log
