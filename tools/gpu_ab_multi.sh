#!/bin/bash
# GPU tests ($TESTS, pytest -k $TESTK), then alternating bench runs of the variants in $VARIANTS
# (";"-separated "ENV=.. ENV2=.. -- bench args" strings), $REPS rounds; summary per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS ${TESTK:+-k "$TESTK"} -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_ab.log; exit 1; }
  tail -3 gpurun_out/pytest_ab.log
fi
: > gpurun_out/ab_bench.log
IFS=';' read -ra VS <<< "$VARIANTS"
for i in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    envs="${v%%--*}"; args="${v#*--}"
    echo "== $v" >> gpurun_out/ab_bench.log
    env FV_X=0 $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 $args >> gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
  done
done
python tools/ab_summary.py gpurun_out/ab_bench.log
grep -o '"host_issue_ms_per_step": [0-9.]*' gpurun_out/ab_bench.log | head -6
grep -o '"families_avg_ms": {[^}]*}' gpurun_out/ab_bench.log | head -3
