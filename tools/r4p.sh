# round-4 session p: small-batch res conv tiles -- parity at B=8, convbench A/B, fbench
cd "$GRAFT_REPO_ROOT"
BASE=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so
TESTS="tests/test_kernels_gpu.py tests/test_warp_gpu.py tests/test_model_gpu.py" bash tools/gpu.sh test || exit 1
CB_ARGS="--layers res,gin --only fwd,dgrad --batch 8 --iters 20" VARIANTS="FV_LIB_PATH=$BASE -- ;-- " REPS=2 bash tools/gpu.sh cbab || exit 1
for v in "$BASE" "" "$BASE" ""; do FV_LIB_PATH=$v timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 >> gpurun_out/fbench_r4p.log || exit 1; done
cat gpurun_out/fbench_r4p.log | cut -c1-200
