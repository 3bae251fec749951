# round-4 session e: 4-wave res conv A/B + parity, full GPU tests, fp8 B=64 A/B, step profile
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
CB_ARGS="--layers res,gin,down2 --only fwd,dgrad --iters 20" VARIANTS="-- ;FV_RES4W=1 -- " REPS=2 bash tools/gpu.sh cbab || exit 1
FV_RES4W=1 TESTS="tests/test_layers_gpu.py tests/test_kernels_gpu.py" TESTK="not fp8" bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4e_res4w.log
VARIANTS="-- ;FV_RES4W=1 -- " REPS=2 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4e_res4w.log
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4e.log
VARIANTS="-- --batch 64 --dtype fp8;FV_FP8_WGRAD=0 -- --batch 64 --dtype fp8;-- --batch 64" REPS=1 bash tools/gpu.sh ab || exit 1
TAG=r4e bash tools/gpu.sh prof
