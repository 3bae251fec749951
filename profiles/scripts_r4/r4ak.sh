# round-4 session ak: out_conv forward with (m-tile, 2 output rows) waves (conv7_n3_fwd3; FV_C7F3=0 = fwd2) -- parity, convbench, step A/B
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_kernels_gpu.py tests/test_layers_gpu.py tests/test_model_gpu.py" TESTK="7 or 256-32 or step" bash tools/gpu.sh test || exit 1
for v in 0 1 0 1; do echo "C7F3=$v"; FV_C7F3=$v timeout -k 10 200 python tools/convbench.py --layers out7 --only fwd --iters 20 2>/dev/null | grep -o '"fwd_us": [0-9.]*' || exit 1; done
for v in 0 1 0 1; do echo "C7F3=$v B=8"; FV_C7F3=$v timeout -k 10 200 python tools/convbench.py --layers out7 --only fwd --iters 20 --batch 8 2>/dev/null | grep -o '"fwd_us": [0-9.]*' || exit 1; done
VARIANTS="FV_C7F3=0 -- ;FV_C7F3=1 -- " REPS=3 bash tools/gpu.sh ab || exit 1
