#!/bin/bash
# Diagnostic build of the decode unit with extra flags into topazdb_amd/variants/libtpz_gpu_NAME.so
# (run here, on the CPU; the .so travels to the GPU box).  tools/build_variant.sh NAME [-DFLAG ...]
set -e
cd "$(dirname "$0")/../topazdb_amd/csrc"
make -s
NAME=$1; shift
mkdir -p build/v_$NAME ../variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-variable \
  -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c tpz_decode.hip -o build/v_$NAME/d.o
/opt/rocm/bin/hipcc -shared -fPIC -Wl,--no-undefined --offload-arch=gfx950 -o ../variants/libtpz_gpu_$NAME.so \
  build/v_$NAME/d.o $(ls build/tpz_*.o | grep -v tpz_decode.o)
