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
