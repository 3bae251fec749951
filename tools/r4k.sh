# round-4 session k: conv3_halo_fwd3 tap-shift (DRV) -- A/B, per-launch parity, step A/B
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
CB_ARGS="--layers res,gin,down2 --only fwd,dgrad --iters 20" VARIANTS="FV_TAPSHIFT=0 -- ;FV_TAPSHIFT=1 -- " REPS=2 bash tools/gpu.sh cbab || exit 1
TESTS="tests/test_layers_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py" bash tools/gpu.sh test || exit 1
VARIANTS="FV_TAPSHIFT=0 -- ;FV_TAPSHIFT=1 -- " REPS=3 bash tools/gpu.sh ab || exit 1
