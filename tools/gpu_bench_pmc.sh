#!/bin/bash
# bench line (with the CPU baseline) + the counter passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
bash tools/gpu_pmc.sh
