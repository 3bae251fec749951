#!/bin/bash
# Config C4 (512x512, B=8): parity tests vs the oracle and a bench line; then the PMC traffic
# passes of the default bench (tools/gpu_pmc.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -k full512 -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_c4.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_c4.log; exit 1; }
grep -E "deviation|passed|failed" gpurun_out/pytest_c4.log
timeout -k 10 300 python bench.py --res 512 --batch 8 --steps 10 --warmup 3 --cpu-seconds 20 > gpurun_out/bench_c4.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c4.log
bash tools/gpu_pmc.sh
