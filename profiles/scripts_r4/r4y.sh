# round-4 session y: depth-reuse conv3d forward as the default -- parity, conv3dbench, fbench + trace
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_afe3d_gpu.py tests/test_warp_gpu.py" bash tools/gpu.sh test || exit 1
for b in 32 16 8; do timeout -k 10 200 python tools/conv3dbench.py --batch $b 2>/dev/null | tail -1 | tee -a gpurun_out/r4y_conv3dbench.jsonl | cut -c1-330 || exit 1; done
for i in 1 2; do timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | tee gpurun_out/r4y_fbench.json | cut -c1-160 || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4y_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/fbench.py" --batch 8 --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/r4y_prof.log" 2>&1
