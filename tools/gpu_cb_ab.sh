#!/bin/bash
# convbench A/B: $CB_ARGS per variant in $VARIANTS (";"-separated env strings), $REPS rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/cb_ab.log
IFS=';' read -ra VS <<< "$VARIANTS"
for i in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    echo "== $v" >> gpurun_out/cb_ab.log
    env FV_X=0 $v timeout -k 10 200 python tools/convbench.py $CB_ARGS >> gpurun_out/cb_ab.log 2>&1 || { tail -20 gpurun_out/cb_ab.log; exit 1; }
  done
done
cat gpurun_out/cb_ab.log | grep -v "^$" | head -80
