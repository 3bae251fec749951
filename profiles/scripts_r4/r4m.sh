# round-4 session m: tests, fold-threshold A/B, conv3d DPP A/B, fbench + its trace
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
BASE=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4m.log
for v in "" "$BASE" "" "$BASE"; do FV_LIB_PATH=$v timeout -k 10 200 python tools/conv3dbench.py >> gpurun_out/conv3dbench_r4m.log 2>&1 || exit 1; done
grep -v amdgpu.ids gpurun_out/conv3dbench_r4m.log
VARIANTS="FV_LIB_PATH=$BASE -- ;-- " REPS=3 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4m_fold.log
timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 > gpurun_out/fbench_r4m.log 2>&1; tail -1 gpurun_out/fbench_r4m.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r4m_fbench -o run -- python3 $GRAFT_REPO_ROOT/tools/fbench.py --batch 8 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_r4m_fbench.log 2>&1) || exit 1
