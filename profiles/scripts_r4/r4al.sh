# round-4 session al: 64-co halo tiles for the latent res convs at small batch (FV_H3BN=64) -- per-launch parity, convbench B=8, fbench
cd "$GRAFT_REPO_ROOT"
FV_H3BN=64 TESTS="tests/test_layers_gpu.py" TESTK="256-32" bash tools/gpu.sh test > /dev/null || { echo test failed; tail -30 gpurun_out/pytest.log; exit 1; }
for v in 0 64 0 64; do echo "H3BN=$v"; FV_H3BN=$v timeout -k 10 200 python tools/convbench.py --layers res --only fwd,dgrad --iters 20 --batch 8 2>/dev/null | grep -o '"fwd_us": [0-9.]*\|"dgrad_us": [0-9.]*' | paste -sd' ' || exit 1; done
for v in 0 64 0 64; do echo "fbench H3BN=$v"; FV_H3BN=$v timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c100-160 || exit 1; done
