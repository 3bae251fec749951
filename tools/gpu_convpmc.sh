#!/bin/bash
# Stall anatomy of the conv kernels: SQ counter passes over tools/convbench.py (LAYERS, ONLY).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C="$R/tools/convbench.py --iters 5 --layers ${LAYERS:-res} --only ${ONLY:-fwd,wgrad}"
cd /tmp
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/cpmc_p$i -o run -- \
    python3 $C > $R/gpurun_out/cpmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/cpmc_p$i.log; exit 1; }
done
cd $R && python tools/pmc_sq.py gpurun_out/cpmc_p1 gpurun_out/cpmc_p2
