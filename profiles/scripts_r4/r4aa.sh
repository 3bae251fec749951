# round-4 session aa: conv3d_c32_fwd_dr with padded rows, every kw fragment from LDS (FV_C3PAD=1) -- parity, A/B
cd "$GRAFT_REPO_ROOT"
FV_C3PAD=1 TESTS="tests/test_afe3d_gpu.py" bash tools/gpu.sh test || exit 1
for b in 32 8; do for r in 1 2; do for v in 0 1; do echo "B=$b PAD=$v"; FV_C3PAD=$v timeout -k 10 200 python tools/conv3dbench.py --batch $b 2>/dev/null | tail -1 | cut -c60-200 || exit 1; done; done; done
for r in 1 2; do for v in 0 1; do echo "fbench PAD=$v"; FV_C3PAD=$v timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c100-160 || exit 1; done; done
