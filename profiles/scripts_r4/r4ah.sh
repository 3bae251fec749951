# round-4 session ah2: BN record folds, two levels over 16-channel segments (FV_FOLD16=2) -- parity, step A/B, trace
cd "$GRAFT_REPO_ROOT"
FV_FOLD16=2 TESTS="tests/test_layers_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_afe3d_gpu.py" TESTK="not 512" bash tools/gpu.sh test || exit 1
VARIANTS="FV_FOLD16=0 -- ;FV_FOLD16=2 -- " REPS=3 bash tools/gpu.sh ab || exit 1
cd /tmp && export TMPDIR=/tmp
FV_FOLD16=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4ah_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/r4ah_prof.log" 2>&1
