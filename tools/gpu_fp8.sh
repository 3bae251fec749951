#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_fp8_gpu.py "tests/test_layers_gpu.py::test_fp8_every_conv_launch_and_step_deviation" > gpurun_out/pytest_fp8.log 2>&1 || { grep -E "Error|FAIL|assert" gpurun_out/pytest_fp8.log | head -20; tail -5 gpurun_out/pytest_fp8.log; exit 1; }
tail -1 gpurun_out/pytest_fp8.log
for B in 32 64; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --dtype fp8 --batch $B > gpurun_out/bench_fp8_$B.log 2>&1 || exit 1; python tools/benchline.py < gpurun_out/bench_fp8_$B.log; done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --batch 64 > gpurun_out/bench_bf16_64.log 2>&1 || exit 1; python tools/benchline.py < gpurun_out/bench_bf16_64.log
