# round-4 session t: fp8 conv with a 3-deep weight ring -- A/B, parity, fp8 step A/B
cd "$GRAFT_REPO_ROOT"
CB_ARGS="--layers res,gin --only fwd,dgrad --batch 64 --dtype fp8 --iters 10" VARIANTS="FV_FP8_NSW3=0 -- ;FV_FP8_NSW3=1 -- " REPS=2 bash tools/gpu.sh cbab > /dev/null || exit 1
grep -o '"layer": "[a-z]*"\|"fp8_fwd_us": [0-9.]*\|"fp8_dgrad_us": [0-9.]*\|== .*' gpurun_out/cbab.log | paste -sd' ' | sed 's/==/\n==/g'
TESTS="tests/test_fp8_gpu.py" bash tools/gpu.sh test || exit 1
TESTS="tests/test_layers_gpu.py" TESTK="fp8" bash tools/gpu.sh test || exit 1
VARIANTS="FV_FP8_NSW3=0 -- --batch 64 --dtype fp8;FV_FP8_NSW3=1 -- --batch 64 --dtype fp8" REPS=2 bash tools/gpu.sh ab || exit 1
