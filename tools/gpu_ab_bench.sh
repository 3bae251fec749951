#!/bin/bash
# alternating bench.py A/B of one env knob on one box: AB_KNOB, AB_REPS, AB_ARGS
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/ab_bench.log
for i in $(seq 1 ${AB_REPS:-3}); do
  for v in "FV_X=0" "$AB_KNOB"; do
    echo "== $v" >> gpurun_out/ab_bench.log
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 ${AB_ARGS:-} >> gpurun_out/ab_bench.log 2>&1 || exit 1
  done
done
