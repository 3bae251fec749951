# round-4 session af: res-conv weight gradient (conv3_halo_wgrad2) with hoisted transposed-read addressing -- parity, A/B
cd "$GRAFT_REPO_ROOT"
TESTS="tests/test_layers_gpu.py" TESTK="wgrad or 256-32" bash tools/gpu.sh test || exit 1
CB_ARGS="--layers res,down2 --only wgrad --iters 20" VARIANTS="-- --lib face-vae_amd/csrc/build_ab/libfacevae_base.so;-- " REPS=2 bash tools/gpu.sh cbab > /dev/null || exit 1
grep -o '"layer": "[a-z0-9]*"\|"wgrad_us": [0-9.]*\|== .*' gpurun_out/cbab.log | paste -sd' ' | sed 's/==/\n==/g'
VARIANTS="FV_LIB_PATH=$GRAFT_REPO_ROOT/face-vae_amd/csrc/build_ab/libfacevae_base.so -- ;FV_LIB_PATH= -- " REPS=2 bash tools/gpu.sh ab || exit 1
