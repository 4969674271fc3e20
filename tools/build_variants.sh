#!/bin/bash
# A/B builds of libmit_hip.so with compile-time kernel switches, for the micro-benchmarks and
# bench.py under MIT_LIB=... . SRC names the source the flags apply to (default gemm; e.g.
# SRC=attention for MIT_ATTN_*); the other objects come from the in-tree build.
# Usage: [SRC=attention] tools/build_variants.sh NAME "-DFOO=1 -DBAR=2" ...
set -e
cd "$(dirname "$0")/../multimodal-image-transformer_amd/csrc"
SRC=${SRC:-gemm}
mkdir -p ../lib/ab build/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c $SRC.hip -o build/variants/${SRC}_$name.o
  objs=""
  for s in capi gemm norm attention misc decode image; do
    if [ $s = $SRC ]; then objs="$objs build/variants/${SRC}_$name.o"; else objs="$objs build/$s.o"; fi
  done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -o ../lib/ab/libmit_hip_$name.so
  echo "built ../lib/ab/libmit_hip_$name.so ($SRC.hip: $flags)"
done
