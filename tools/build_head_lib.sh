#!/bin/bash
# A/B helper: build libfacevae.so from a committed conv.hip (default HEAD) into abl/libfacevae_<tag>.so,
# linking this tree's other objects (run after face-vae_amd/csrc/build.py).
#   bash tools/build_head_lib.sh [rev] [tag]
set -e
REV=${1:-HEAD}; TAG=${2:-head}
cd "$(dirname "$0")/.."
git show "$REV":face-vae_amd/csrc/conv.hip > face-vae_amd/csrc/conv_ab_tmp.hip
(cd face-vae_amd/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -mcode-object-version=5 \
   -I../../include -c conv_ab_tmp.hip -o /tmp/conv_ab_tmp.o) || { rm -f face-vae_amd/csrc/conv_ab_tmp.hip; exit 1; }
rm -f face-vae_amd/csrc/conv_ab_tmp.hip
mkdir -p abl
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libfacevae_$TAG.so /tmp/conv_ab_tmp.o \
  $(ls face-vae_amd/csrc/build/*.o | grep -v conv.hip.o) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built abl/libfacevae_$TAG.so from $REV"
