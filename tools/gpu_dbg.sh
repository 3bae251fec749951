#!/bin/bash
# v2 forward knob sweep (FV_CONV_DBG bits: 1 skip MFMA [ref loop], 2 skip DMA, 4 skip epilogue, 8 ref loop)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
rm -f gpurun_out/dbg.log
for d in ${DBGS:-0 2 4 6 8 9 13}; do
  echo "== FV_CONV_DBG=$d" >> gpurun_out/dbg.log
  FV_CONV_DBG=$d timeout -k 10 200 python tools/convbench.py --layers ${LAYERS:-res,down1,up2} --only fwd --iters 20 >> gpurun_out/dbg.log 2>&1 || exit 1
done
