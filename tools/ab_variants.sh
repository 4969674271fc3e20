#!/bin/bash
# run tools/gemm_bench.py against several A/B builds (tools/build_variants.sh), twice, alternating
set -o pipefail
for rep in 1 2; do
for v in "$@"; do
  echo "== $v" >> gpurun_out/ab.log
  MIT_LIB=multimodal-image-transformer_amd/lib/variants/libmit_hip_$v.so timeout -k 10 100 python tools/gemm_bench.py 2 >> gpurun_out/ab.log 2>&1 || exit 1
done
done
