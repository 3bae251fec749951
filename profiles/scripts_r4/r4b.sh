# round-4 session b: wgrad kernel A/B, step A/B of the two changes, GPU tests, kernel trace
cd "$GRAFT_REPO_ROOT"
export TAG=r4b TEST_TIMEOUT=800
CB_ARGS="--layers res,gin,down2,down1 --only wgrad --iters 20" VARIANTS="FV_H3W_ALL=0 -- ;FV_H3W_ALL=1 -- " REPS=2 \
  bash tools/gpu.sh cbab || exit 1
VARIANTS="FV_NAC_STAGED=0 FV_H3W_ALL=0 -- ;FV_NAC_STAGED=0 FV_H3W_ALL=1 -- ;FV_NAC_STAGED=1 FV_H3W_ALL=1 -- " REPS=2 \
  bash tools/gpu.sh ab || exit 1
bash tools/gpu.sh test prof
