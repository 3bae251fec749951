# round-4 session x: depth-reuse conv3d forward (FV_C3DR=1, FV_C3XCD=1) -- parity under the knobs, A/B
cd "$GRAFT_REPO_ROOT"
FV_C3DR=1 FV_C3XCD=1 TESTS="tests/test_afe3d_gpu.py" bash tools/gpu.sh test || exit 1
for b in 32 8; do for r in 1 2; do for v in "0 0" "1 0" "1 1"; do set -- $v; echo "B=$b DR=$1 XCD=$2"; FV_C3DR=$1 FV_C3XCD=$2 timeout -k 10 200 python tools/conv3dbench.py --batch $b 2>/dev/null | tail -1 | cut -c1-330 || exit 1; done; done; done
for r in 1 2; do for v in "0 0" "1 1"; do set -- $v; echo "fbench DR=$1 XCD=$2"; FV_C3DR=$1 FV_C3XCD=$2 timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c1-160 || exit 1; done; done
