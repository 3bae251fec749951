# round-4 session s: fp8 B=64 step trace (and bf16 B=64 for comparison)
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--batch 64 --dtype fp8" TAG=r4s_fp8_b64 bash tools/gpu.sh prof || exit 1
BENCH_ARGS="--batch 64" TAG=r4s_bf16_b64 bash tools/gpu.sh prof || exit 1
