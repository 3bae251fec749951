# round-4 session h: fp8 unit tests (wgrad operand classes, subnormals)
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_fp8_gpu.py" bash tools/gpu.sh test; cp gpurun_out/pytest.log gpurun_out/pytest_r4h_fp8.log
grep -E "fp8 wgrad|fp8 conv" gpurun_out/pytest.log
