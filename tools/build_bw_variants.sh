#!/bin/bash
# Build bigwave pipeline-shape variants (tools/abl_multi.py names them bw_<name>):
#   tools/build_bw_variants.sh name:"flags" ...
set -e
cd "$(dirname "$0")/../topazdb_amd/csrc"
make -s -j8 >/dev/null
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p build/$name ../variants
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-variable $flags -c tpz_bigwave.hip -o build/$name/b.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../variants/libtpz_gpu_$name.so build/tpz_decode.o build/$name/b.o build/tpz_crc.o build/tpz_codec.o build/tpz_seek.o build/tpz_spill.o build/tpz_api.o build/tpz_host_pipeline.o build/tpz_host_builder.o
done
