# round-4 session aj: level 2 of the record folds by one thread per channel (fold_rows_kernel; FV_FOLD_ROWS=0 = fold1) -- parity, A/B, trace
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_layers_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py" TESTK="not 512" bash tools/gpu.sh test || exit 1
VARIANTS="FV_FOLD_ROWS=0 -- ;FV_FOLD_ROWS=1 -- " REPS=3 bash tools/gpu.sh ab || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4aj_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/r4aj_prof.log" 2>&1
