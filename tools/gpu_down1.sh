#!/bin/bash
# down1 / down2 conv variants (halo pipelined vs single-tap, v2) at the B=32 shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { echo "== $1" >> gpurun_out/down1.log; env $1 timeout -k 10 200 python tools/convbench.py --layers down1,down2,up2 --only fwd,dgrad >> gpurun_out/down1.log 2>&1 || exit 1; }
run "FV_X=0"
run "FV_H3_PIPE=1"
run "FV_DISABLE_H3=1"
