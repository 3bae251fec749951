#!/bin/bash
# per-layer conv timings under the path knobs (one box, back to back)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/sweep.log
for v in "FV_X=0" "FV_DISABLE_H3=1" "FV_H3_PIPE=0" "FV_H3SUB=1" "FV_DISABLE_H3W=1" "FV_DISABLE_SUBPIX=1" "FV_V2_CFG=4"; do
  echo "== $v" >> gpurun_out/sweep.log
  env $v timeout -k 10 200 python tools/convbench.py >> gpurun_out/sweep.log 2>&1 || exit 1
done
