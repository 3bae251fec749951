#!/bin/bash
# end-of-session verification: smoke(), every GPU test, the default bench and a rocprof summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
TAG=${TAG:-verify} bash tools/gpu_prof.sh || exit 1
tail -2 gpurun_out/pytest_gpu.log
tail -1 gpurun_out/bench.log | cut -c1-420
