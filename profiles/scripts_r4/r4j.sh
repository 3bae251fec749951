# round-4 session j: coalesced chunked BN fold -- GPU tests, step A/B against the previous fold, profile
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4j.log
VARIANTS="-- ;FV_LIB_PATH=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so -- " REPS=3 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4j_fold.log
TAG=r4j bash tools/gpu.sh prof
