# round-4 session g: fp8 wgrad / subnormal probes, then the full GPU tests, fp8 A/B, step profile
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
TESTS="tests/test_fp8_gpu.py" bash tools/gpu.sh test; cp gpurun_out/pytest.log gpurun_out/pytest_r4g_fp8.log
TESTS="tests/test_layers_gpu.py" TESTK="fp8" bash tools/gpu.sh test; cp gpurun_out/pytest.log gpurun_out/pytest_r4g_layers8.log
FV_FP8_WGRAD=0 TESTS="tests/test_layers_gpu.py" TESTK="fp8" bash tools/gpu.sh test; cp gpurun_out/pytest.log gpurun_out/pytest_r4g_layers8_nowg.log
VARIANTS="-- --batch 64 --dtype fp8;FV_FP8_WGRAD=0 -- --batch 64 --dtype fp8;-- --batch 64" REPS=1 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4g_fp8.log
TAG=r4g bash tools/gpu.sh prof
