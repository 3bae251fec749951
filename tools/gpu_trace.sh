#!/bin/bash
# Kernel-trace profile of the bench (tests skipped): per-step trace + stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-it}
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench.log 2>&1 || exit 1
python tools/benchline.py < gpurun_out/bench.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
