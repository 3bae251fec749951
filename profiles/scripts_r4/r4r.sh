# round-4 session r: ResBlock BN-backward sums in the dgrad store pass (FV_RES_SR) -- parity, step A/B
cd "$GRAFT_REPO_ROOT"
FV_RES_SR=1 TESTS="tests/test_layers_gpu.py" TESTK="not fp8 and not nac" bash tools/gpu.sh test || exit 1
VARIANTS="FV_RES_SR=0 -- ;FV_RES_SR=1 -- " REPS=3 bash tools/gpu.sh ab || exit 1
