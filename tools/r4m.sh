# round-4 session m: fold threshold A/B, tests, counters (r4_pmc), profile
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
BASE=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4m.log
VARIANTS="FV_LIB_PATH=$BASE -- ;-- " REPS=3 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4m_fold.log
bash tools/gpu.sh pmc || exit 1
cp gpurun_out/pmc.json gpurun_out/pmc_r4m.json
CB_ARGS="--layers res --only fwd,wgrad --iters 5" bash tools/gpu.sh convpmc || exit 1
cp gpurun_out/convpmc.txt gpurun_out/convpmc_r4m_res.txt
TAG=r4m bash tools/gpu.sh prof
TESTS="tests/test_afe3d_gpu.py tests/test_warp_gpu.py" bash tools/gpu.sh test || exit 1
for v in "" "$BASE"; do FV_LIB_PATH=$v timeout -k 10 200 python tools/conv3dbench.py >> gpurun_out/conv3dbench_r4m.log 2>&1 || exit 1; done
for v in "" "$BASE"; do FV_LIB_PATH=$v timeout -k 10 200 python tools/conv3dbench.py >> gpurun_out/conv3dbench_r4m.log 2>&1 || exit 1; done
grep -v amdgpu.ids gpurun_out/conv3dbench_r4m.log
timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 > gpurun_out/fbench_r4m.log 2>&1; tail -1 gpurun_out/fbench_r4m.log
