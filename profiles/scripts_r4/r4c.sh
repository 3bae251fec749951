# round-4 session c: tr_b8 probe, staged-NAC kernels vs plain, step A/B, fp8 weight gradient
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
TESTS="tests/test_fp8_gpu.py" TESTK="tr8" bash tools/gpu.sh test || exit 1
CB_ARGS="--layers res --only fwd,wgrad --iters 20" VARIANTS="-- ;-- --pro" REPS=2 bash tools/gpu.sh cbab || exit 1
CB_ARGS="--layers res,down2 --only fwd,dgrad,wgrad --batch 64 --dtype fp8 --iters 10" bash tools/gpu.sh convbench || exit 1
VARIANTS="FV_NAC_STAGED=0 -- ;FV_NAC_STAGED=1 -- " REPS=2 bash tools/gpu.sh ab || exit 1
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4c.log
VARIANTS="-- --batch 64 --dtype fp8;FV_FP8_WGRAD=0 -- --batch 64 --dtype fp8;-- --batch 64" REPS=1 bash tools/gpu.sh ab || exit 1
TAG=r4c bash tools/gpu.sh prof
