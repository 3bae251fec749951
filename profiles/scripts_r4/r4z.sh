# round-4 session z: XCD-grouped block order for conv3d_c32_fwd_dr -- fbench A/B, conv3dbench
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do for v in 0 1; do echo "fbench XCD=$v"; FV_C3XCD=$v timeout -k 10 300 python tools/fbench.py --batch 8 --steps 10 --warmup 3 2>/dev/null | tail -1 | cut -c100-160 || exit 1; done; done
for b in 32 8; do for v in 0 1; do echo "B=$b XCD=$v"; FV_C3XCD=$v timeout -k 10 200 python tools/conv3dbench.py --batch $b 2>/dev/null | tail -1 | cut -c60-130 || exit 1; done; done
