# round-4 session k: conv3_halo_fwd3 tap-shift (DRV) and the octet BN fold -- A/B, parity, step A/B
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
BASE=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so
CB_ARGS="--layers res,gin,down2 --only fwd,dgrad --iters 20" VARIANTS="FV_TAPSHIFT=0 -- ;FV_TAPSHIFT=1 -- " REPS=2 bash tools/gpu.sh cbab || exit 1
timeout -k 10 200 python tools/bnbench.py > gpurun_out/bnbench_k.log 2>&1 && FV_LIB_PATH=$BASE timeout -k 10 200 python tools/bnbench.py >> gpurun_out/bnbench_k.log 2>&1 || exit 1
cat gpurun_out/bnbench_k.log
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4k.log
VARIANTS="FV_TAPSHIFT=0 FV_LIB_PATH=$BASE -- ;FV_TAPSHIFT=1 FV_LIB_PATH=$BASE -- ;FV_TAPSHIFT=1 -- " REPS=3 bash tools/gpu.sh ab || exit 1
cp gpurun_out/ab.log gpurun_out/ab_r4k.log
TAG=r4k bash tools/gpu.sh prof
CB_ARGS="--layers down1 --only dgrad --iters 5" TAG=r4k_down1 bash tools/gpu.sh convpmc
timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 > gpurun_out/fbench_r4k.log 2>&1; tail -2 gpurun_out/fbench_r4k.log
timeout -k 10 300 python tools/databench.py > gpurun_out/databench_r4k.log 2>&1; tail -1 gpurun_out/databench_r4k.log
