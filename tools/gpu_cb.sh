#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/convbench.py $CB_ARGS > gpurun_out/cb.log 2>&1 || { tail -20 gpurun_out/cb.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cb.log
