#!/bin/bash
# Conv tile sweep on the GPU box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in -1 3 4 5; do
  echo "== FV_V2_CFG=$cfg" >> gpurun_out/convbench.log
  FV_V2_CFG=$cfg timeout -k 10 300 python tools/convbench.py --only fwd,dgrad,wgrad >> gpurun_out/convbench.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/bench2.log 2>&1
