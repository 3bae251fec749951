set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
{ nproc; python -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo OMP=$OMP_NUM_THREADS; } > gpurun_out/probe.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_layers_gpu.py tests/test_train_gpu.py -s > gpurun_out/pytest_new.log 2>&1
