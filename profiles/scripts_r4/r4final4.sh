# round-4 final session 4 (after the conv3d epilogue switches and the one-lane gather): full GPU tests, smoke, default bench (with CPU baseline), step profile, other configs
cd "$GRAFT_REPO_ROOT"
export TEST_TIMEOUT=900
bash tools/gpu.sh test || exit 1
cp gpurun_out/pytest.log gpurun_out/pytest_r4final4.log
bash tools/gpu.sh smoke || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_r4final4.log 2>&1 || { tail -20 gpurun_out/bench_r4final4.log; exit 1; }
tail -1 gpurun_out/bench_r4final4.log | cut -c1-300
TAG=r4final4 bash tools/gpu.sh prof || exit 1
bash tools/gpu.sh configs
timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 > gpurun_out/fbench_r4final4.json || exit 1
