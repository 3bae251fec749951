# round-4 session i: fp8 tests, full GPU tests, fp8 B=64 A/B, step profile
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
TESTS="tests/test_fp8_gpu.py" bash tools/gpu.sh test || exit 1
grep -E "fp8 wgrad|fp8 MFMA" gpurun_out/pytest.log
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4i.log
VARIANTS="-- --batch 64 --dtype fp8;FV_FP8_WGRAD=0 -- --batch 64 --dtype fp8;-- --batch 64" REPS=2 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4i_fp8.log
TAG=r4i bash tools/gpu.sh prof
