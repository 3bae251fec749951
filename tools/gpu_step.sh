#!/bin/bash
# One box session: named tests (TESTS, default all -m gpu), then optional bench lines (BENCHES:
# ';'-separated bench.py argument lists) and an optional rocprofv3 kernel-trace of PROF_ARGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread ${TESTS:-tests -m gpu} \
  > gpurun_out/pytest_step.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_step.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_step.log | head -20; tail -3 gpurun_out/pytest_step.log; exit 1; }
tail -2 gpurun_out/pytest_step.log
i=0
IFS=';' read -ra BL <<< "${BENCHES:-}"
for b in "${BL[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 $b > gpurun_out/bench_$i.log 2>&1 || exit 1
  echo "[$b]"; python tools/benchline.py < gpurun_out/bench_$i.log
done
if [ -n "$PROF_ARGS" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG:-x} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 $PROF_ARGS > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG:-x}.log 2>&1 || exit 1
fi
