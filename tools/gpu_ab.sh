#!/bin/bash
# alternating A/B of one knob on selected layers: AB_KNOB, AB_LAYERS, AB_ONLY, AB_REPS
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/ab.log
for i in $(seq 1 ${AB_REPS:-3}); do
  for v in "FV_X=0" "$AB_KNOB"; do
    echo "== $v" >> gpurun_out/ab.log
    env $v timeout -k 10 200 python tools/convbench.py --layers $AB_LAYERS --only $AB_ONLY >> gpurun_out/ab.log 2>&1 || exit 1
  done
done
