# round-4 session n: counters (r4_pmc), res conv SQ passes, step profile
cd "$GRAFT_REPO_ROOT"
bash tools/gpu.sh pmc || exit 1
cp gpurun_out/pmc.json gpurun_out/pmc_r4n.json
CB_ARGS="--layers res --only fwd,wgrad --iters 5" bash tools/gpu.sh convpmc || exit 1
cp gpurun_out/convpmc.txt gpurun_out/convpmc_r4n_res.txt
TAG=r4n bash tools/gpu.sh prof
