# round-4 session ao: grid-sample input-gradient gather, one lane per 32-channel cell (FV_GS_WHOLE=0: 4 lanes) -- parity, fbench A/B, trace
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_warp_gpu.py" bash tools/gpu.sh test || exit 1
for r in 1 2; do for v in 0 1; do echo "fbench WHOLE=$v"; FV_GS_WHOLE=$v timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c100-160 || exit 1; done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4ao_prof" -o run -- python3 "$GRAFT_REPO_ROOT/tools/fbench.py" --batch 8 --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/r4ao_prof.log" 2>&1
