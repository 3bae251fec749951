#!/bin/bash
# Counters of the bench's kernels: a --kernel-trace --stats run, then one rocprofv3 --pmc pass
# per counter group (FETCH_SIZE; WRITE_SIZE; SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE), each
# its own short bench run; then tools/pmc_collect.py -> gpurun_out/pmc.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 2 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-}"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc_trace -o run -- \
  python3 $B > $R/gpurun_out/pmc_trace.log 2>&1 || { echo "trace failed"; tail -5 $R/gpurun_out/pmc_trace.log; exit 1; }
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_p$i -o run -- \
    python3 $B > $R/gpurun_out/pmc_p$i.log 2>&1 || { echo "pmc $c failed"; tail -5 $R/gpurun_out/pmc_p$i.log; exit 1; }
done
cd $R && python tools/pmc_collect.py --trace gpurun_out/pmc_trace --pass gpurun_out/pmc_p1 --pass gpurun_out/pmc_p2 \
  --pass gpurun_out/pmc_p3 > gpurun_out/pmc.json && python -c "
import json; d=json.load(open('gpurun_out/pmc.json'))
for k,v in d['dominant'].items(): print(k, {a: (round(b,4) if isinstance(b,float) else b) for a,b in v.items() if a!='kernel'})
print('step', d['step'])"
