#!/bin/bash
# build libgibbs_hip.so variants with extra -D flags into build_variants/ (CPU side)
# usage: tools/build_variants.sh NAME "-DFLAG1 -DFLAG2" [NAME2 "FLAGS2" ...]
set -e
cd "$(dirname "$0")/.."
mkdir -p build_variants
S=gibbssampler_amd/csrc
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  hipcc --offload-arch=gfx950 -O3 -ffp-contract=on -std=c++17 -shared -fPIC -I include $flags \
    -o build_variants/lib_$name.so $S/gs_kernels.hip $S/gs_sht.hip $S/gs_masked.hip &
done
wait
