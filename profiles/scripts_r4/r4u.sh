# round-4 session u: conv3d weight gradient depth chunks at small batch -- parity, fbench
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_afe3d_gpu.py tests/test_warp_gpu.py" bash tools/gpu.sh test || exit 1
for b in 8 32; do timeout -k 10 200 python tools/conv3dbench.py --batch $b 2>/dev/null | tail -1; done
for i in 1 2; do timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c1-200; done
