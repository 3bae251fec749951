#!/bin/bash
# HBM traffic of the bench's kernels: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; they
# do not fit one pass), each its own short bench run; then tools/pmc_traffic.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_$c -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $R/gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $R/gpurun_out/pmc_$c.log; exit 1; }
done
cd $R && python tools/pmc_traffic.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc_traffic.json && cat gpurun_out/pmc_traffic.json
