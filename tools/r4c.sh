# round-4 session c: staged-NAC kernels vs plain (convbench), step A/B, GPU tests, kernel traces
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=800
CB_ARGS="--layers res --only fwd,wgrad --iters 20" VARIANTS="-- ;-- --pro" REPS=2 bash tools/gpu.sh cbab || exit 1
VARIANTS="FV_NAC_STAGED=0 -- ;FV_NAC_STAGED=1 -- " REPS=2 bash tools/gpu.sh ab || exit 1
bash tools/gpu.sh test || exit 1
TAG=r4c BENCH_ARGS="" bash tools/gpu.sh prof || exit 1
FV_NAC_STAGED=0 TAG=r4c_nac0 bash tools/gpu.sh prof
