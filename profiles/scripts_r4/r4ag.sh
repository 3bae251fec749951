# round-4 session ag: fp8 weight gradient with 4 row-pair groups in flight (FV_W8_AHEAD=4) -- parity, A/B
cd "$GRAFT_REPO_ROOT"
FV_W8_AHEAD=4 TESTS="tests/test_fp8_gpu.py" TESTK="wgrad" bash tools/gpu.sh test || exit 1
CB_ARGS="--layers res --only wgrad --batch 64 --dtype fp8 --iters 10" VARIANTS="FV_W8_AHEAD=3 -- ;FV_W8_AHEAD=4 -- " REPS=2 bash tools/gpu.sh cbab > /dev/null || exit 1
grep -o '"layer": "[a-z0-9]*"\|"fp8_wgrad_us": [0-9.]*\|"wgrad_us": [0-9.]*\|== .*' gpurun_out/cbab.log | paste -sd' ' | sed 's/==/\n==/g'
VARIANTS="FV_W8_AHEAD=3 -- --batch 64 --dtype fp8;FV_W8_AHEAD=4 -- --batch 64 --dtype fp8" REPS=2 bash tools/gpu.sh ab || exit 1
