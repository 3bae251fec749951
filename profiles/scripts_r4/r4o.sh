# round-4 session o: conv3d 8-wave split A/B + parity; counters (r4_pmc), res conv SQ passes, step profile
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_afe3d_gpu.py tests/test_warp_gpu.py" bash tools/gpu.sh test || exit 1
for v in 0 1 0 1; do FV_C3SPLIT=$v timeout -k 10 200 python tools/conv3dbench.py >> gpurun_out/conv3dbench_r4o.log 2>&1 || exit 1; done
grep -v amdgpu.ids gpurun_out/conv3dbench_r4o.log
bash tools/r4n.sh
