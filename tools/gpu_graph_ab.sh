#!/bin/bash
# new GPU tests (graph / side stream), then an alternating bench A/B: --graph 1 vs --graph 0
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_graph_gpu.py} -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_graph.log; exit 1; }
tail -8 gpurun_out/pytest_graph.log
: > gpurun_out/ab_bench.log
for i in 1 2 3; do
  for v in 1 0; do
    echo "== graph=$v" >> gpurun_out/ab_bench.log
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --graph $v >> gpurun_out/ab_bench.log 2>&1 || exit 1
  done
done
python tools/ab_summary.py gpurun_out/ab_bench.log
grep -o '"host_issue_ms_per_step": [0-9.]*\|"roofline": {[^}]*}' gpurun_out/ab_bench.log | head -4
