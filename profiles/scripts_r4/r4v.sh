# round-4 session v: LDS-tiled bf16 depth split/merge (C=32, D=16) -- parity, fbench, trace
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_afe3d_gpu.py tests/test_warp_gpu.py" bash tools/gpu.sh test || exit 1
for i in 1 2; do timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c1-200 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4v_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/fbench.py" --batch 8 --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/r4v_prof.log" 2>&1
