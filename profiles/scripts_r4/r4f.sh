# round-4 session f: full GPU tests, fp8 B=64 A/B, step profile
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4f.log
VARIANTS="-- --batch 64 --dtype fp8;FV_FP8_WGRAD=0 -- --batch 64 --dtype fp8;-- --batch 64" REPS=1 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4f_fp8.log
TAG=r4f bash tools/gpu.sh prof
