# round-4 session l: pipelined fp8 conv, hybrid fold -- parity, A/B, profile
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
BASE=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so
TESTS="tests/test_fp8_gpu.py" bash tools/gpu.sh test || exit 1
CB_ARGS="--layers res,gin --only fwd,dgrad --batch 64 --dtype fp8 --iters 10" VARIANTS="FV_FP8P=0 -- ;FV_FP8P=1 -- " REPS=2 bash tools/gpu.sh cbab || exit 1
timeout -k 10 200 python tools/bnbench.py > gpurun_out/bnbench_l.log 2>&1 && FV_LIB_PATH=$BASE timeout -k 10 200 python tools/bnbench.py >> gpurun_out/bnbench_l.log 2>&1 || exit 1
cat gpurun_out/bnbench_l.log
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4l.log
VARIANTS="FV_LIB_PATH=$BASE -- ;-- " REPS=3 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4l_fold.log
VARIANTS="FV_FP8P=0 -- --batch 64 --dtype fp8;-- --batch 64 --dtype fp8;-- --batch 64" REPS=2 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4l_fp8.log
TAG=r4l bash tools/gpu.sh prof
