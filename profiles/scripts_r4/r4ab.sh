# round-4 session ab: conv3d_c32_fwd_dr with a 3-slot ring (slices prefetched two steps ahead) -- parity, A/B vs the 2-slot build
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_afe3d_gpu.py" bash tools/gpu.sh test || exit 1
BASE=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so
for b in 32 8; do for r in 1 2; do for v in base new; do echo "B=$b $v"; if [ $v = base ]; then L=$BASE; else L=; fi; FV_LIB_PATH=$L timeout -k 10 200 python tools/conv3dbench.py --batch $b 2>/dev/null | tail -1 | cut -c60-200 || exit 1; done; done; done
for r in 1 2; do for v in base new; do echo "fbench $v"; if [ $v = base ]; then L=$BASE; else L=; fi; FV_LIB_PATH=$L timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c100-160 || exit 1; done; done
