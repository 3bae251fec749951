#!/bin/bash
# GPU tests, an alternating bench A/B of one knob (AB_KNOB) and a kernel-trace profile of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-it}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
fi
if [ -n "$AB_KNOB" ]; then
  : > gpurun_out/ab_bench.log
  for i in $(seq 1 ${AB_REPS:-3}); do
    for v in "FV_X=0" "$AB_KNOB"; do
      echo "== $v" >> gpurun_out/ab_bench.log
      env $v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 ${AB_ARGS:-} >> gpurun_out/ab_bench.log 2>&1 || exit 1
    done
  done
  python tools/ab_summary.py gpurun_out/ab_bench.log
fi
if [ -z "$SKIP_PROF" ]; then
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
fi
