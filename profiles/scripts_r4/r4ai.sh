# round-4 session ai: 16-channel folds as the default (fp32 records: two levels at any size) -- parity, step A/B vs HEAD~, fbench, trace
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_layers_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_afe3d_gpu.py tests/test_distributed_gpu.py" TESTK="not 512" bash tools/gpu.sh test || exit 1
VARIANTS="FV_LIB_PATH=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so -- ;FV_LIB_PATH= -- " REPS=3 bash tools/gpu.sh ab || exit 1
for v in base new; do if [ $v = base ]; then L=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so; else L=; fi; echo "fbench $v"; FV_LIB_PATH=$L timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c100-160 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4ai_prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/r4ai_prof.log" 2>&1
