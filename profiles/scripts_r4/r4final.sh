# round-4 final session: full GPU tests, smoke, default bench (with CPU baseline), step profile, other configs
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4final.log
bash tools/gpu.sh smoke || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_r4final.log 2>&1 || { tail -20 gpurun_out/bench_r4final.log; exit 1; }
tail -1 gpurun_out/bench_r4final.log | cut -c1-300
TAG=r4final bash tools/gpu.sh prof || exit 1
bash tools/gpu.sh configs
