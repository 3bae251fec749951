# round-4 session ad: weight images sized for the v2 co tiles (wrows) -- the faulting AFE case, conv kernels, 3-D trunk
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_afe3d_gpu.py tests/test_kernels_gpu.py tests/test_warp_gpu.py tests/test_graph_gpu.py" bash tools/gpu.sh test || exit 1
for i in 1 2; do timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | tee gpurun_out/r4ac_fbench.json | cut -c100-160 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4ac_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/fbench.py" --batch 8 --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/r4ac_prof.log" 2>&1
