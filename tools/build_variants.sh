#!/bin/bash
# A/B builds of libmit_hip.so with compile-time kernel switches (gemm.hip MIT_G256_*), for
# tools/gemm_bench.py under MIT_LIB=... . Usage: tools/build_variants.sh NAME "-DFOO=1 -DBAR=2" ...
set -e
cd "$(dirname "$0")/../multimodal-image-transformer_amd/csrc"
mkdir -p ../lib/variants build/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c gemm.hip -o build/variants/gemm_$name.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build/capi.o build/variants/gemm_$name.o build/norm.o build/attention.o build/misc.o build/decode.o build/image.o -o ../lib/variants/libmit_hip_$name.so
  echo "built ../lib/variants/libmit_hip_$name.so ($flags)"
done
