# round-4 session p: small-batch res conv tiles -- parity, convbench A/B at B=8, fbench
cd "$GRAFT_REPO_ROOT"
BASE=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so
TESTS="tests/test_kernels_gpu.py tests/test_warp_gpu.py tests/test_model_gpu.py" bash tools/gpu.sh test || exit 1
CB_ARGS="--layers res,gin --only fwd,dgrad --batch 8 --iters 20" VARIANTS="FV_LIB_PATH=$BASE -- ;-- " REPS=2 bash tools/gpu.sh cbab || exit 1
for i in 1 2; do timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 >> gpurun_out/fbench_r4p.log || exit 1; done
cut -c1-200 gpurun_out/fbench_r4p.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r4p_fbench -o run -- python3 $GRAFT_REPO_ROOT/tools/fbench.py --batch 8 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_r4p_fbench.log 2>&1) || exit 1
