# round-4 session q: register-staged weight stages in the res conv (RSW) -- A/B, parity, step A/B
cd "$GRAFT_REPO_ROOT"
CB_ARGS="--layers res,gin --only fwd,dgrad --iters 20" VARIANTS="FV_RSW=0 -- ;FV_RSW=1 -- " REPS=2 bash tools/gpu.sh cbab || exit 1
TESTS="tests/test_layers_gpu.py tests/test_kernels_gpu.py" TESTK="not fp8" bash tools/gpu.sh test || exit 1
VARIANTS="FV_RSW=0 -- ;FV_RSW=1 -- " REPS=3 bash tools/gpu.sh ab || exit 1
