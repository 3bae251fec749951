# round-4 session am: one-launch fp32 record fold with 16-B lanes (fold16v_kernel, FV_FOLDV=1) -- parity, step A/B, trace
cd "$GRAFT_REPO_ROOT"
FV_FOLDV=1 TESTS="tests/test_layers_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py" TESTK="not 512" bash tools/gpu.sh test || exit 1
VARIANTS="FV_FOLDV=0 -- ;FV_FOLDV=1 -- " REPS=3 bash tools/gpu.sh ab || exit 1
cd /tmp && export TMPDIR=/tmp
FV_FOLDV=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4am_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/r4am_prof.log" 2>&1
