#!/bin/bash
# A/B helper: build libfacevae.so from a committed source (default conv.hip at HEAD) into
# abl/libfacevae_<tag>.so, linking this tree's other objects (run after face-vae_amd/csrc/build.py).
#   bash tools/build_head_lib.sh [rev] [tag] [file]      e.g.  bash tools/build_head_lib.sh HEAD head bn.hip
set -e
REV=${1:-HEAD}; TAG=${2:-head}; SRC=${3:-conv.hip}
cd "$(dirname "$0")/.."
git show "$REV":face-vae_amd/csrc/$SRC > face-vae_amd/csrc/ab_tmp_$SRC
(cd face-vae_amd/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -mcode-object-version=5 \
   -I../../include -x hip -c ab_tmp_$SRC -o /tmp/ab_tmp.o) || { rm -f face-vae_amd/csrc/ab_tmp_$SRC; exit 1; }
rm -f face-vae_amd/csrc/ab_tmp_$SRC
mkdir -p abl
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libfacevae_$TAG.so /tmp/ab_tmp.o \
  $(ls face-vae_amd/csrc/build/*.o | grep -v "/$SRC.o") -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built abl/libfacevae_$TAG.so from $REV:$SRC"
