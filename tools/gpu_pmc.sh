#!/bin/bash
# PMC counter passes (separate rocprofv3 runs, kernel-trace only) over a convbench slice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${PMC_ARGS:---layers res --only fwd,dgrad,wgrad --iters 3}
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/tools/convbench.py $ARGS > $GRAFT_REPO_ROOT/gpurun_out/pmc$i.log 2>&1 || exit 1
done
