#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for d in 0 4 1 5 3 7 2 6; do
  echo "== FV_CONV_DBG=$d" >> gpurun_out/dbg.log
  FV_CONV_DBG=$d timeout -k 10 200 python tools/convbench.py --layers res --only fwd --iters 30 >> gpurun_out/dbg.log 2>&1 || exit 1
done
