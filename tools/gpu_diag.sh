#!/bin/bash
# Diagnostics: per-layer conv timings, res-fwd knob sweep (skip MFMA / DMA / epilogue), PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/convbench.py > gpurun_out/convbench_all.log 2>&1 || exit 1
for d in 0 1 2 4 5; do
  echo "== FV_CONV_DBG=$d" >> gpurun_out/dbg.log
  FV_CONV_DBG=$d timeout -k 10 120 python tools/convbench.py --layers res,down1,up2 --only fwd --iters 20 >> gpurun_out/dbg.log 2>&1 || exit 1
done
PMC_ARGS="--layers res,down1,up2,out7,in7 --only fwd,dgrad,wgrad --iters 2" bash tools/gpu_pmc.sh || exit 1
