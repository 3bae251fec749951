#!/bin/bash
# round-end style session: all GPU tests, default bench, rocprof summary, then the other
# BASELINE configs on one GPU (512x512 B=8; B=64 bf16 / fp8 = config C5's per-GPU shard)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-final}
bash tools/gpu_prof.sh || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --res 512 --batch 8 > gpurun_out/bench_c4.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --batch 64 > gpurun_out/bench_b64.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --batch 64 --dtype fp8 > gpurun_out/bench_fp8.log 2>&1 || exit 1
for f in bench bench_c4 bench_b64 bench_fp8; do tail -1 gpurun_out/$f.log | cut -c1-300; done
