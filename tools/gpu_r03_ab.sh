#!/bin/bash
# Round-3 A/Bs, run on the GPU box from the repo root; each arm in its own process,
# arms interleaved. Usage: bash tools/gpu_r03_ab.sh [stage|persist|tall|grouped|nowait|stamps]
#   stage    MIT_G256_STAGE=0/1/2 (register exchange / staged without operands / staged everywhere)
#   persist  MIT_G256_PERSIST=0/1 (one-tile grid / persistent gemm256p_kernel), kernels and the step
#   tall     GEMM variants 2 vs 7 (256x256 vs the two-workgroup 256x128 kernel)
#   grouped  MIT_GROUPED_GROUP=8/1 (grouped dW tile order), the step
#   nowait   the DMA-wait diagnostic build vs the shipped one (tools/build_variants.sh nowait -DMIT_G256_DIAG_NOWAIT)
#   stamps   per-phase clock stamps (tools/build_variants.sh stamp -DMIT_G256_STAMP)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=multimodal-image-transformer_amd/lib/variants
SH="enc_qkv+bias,enc_o+res,enc_fc1+gelu,enc_fc1,enc_fc2+res,dec_kv_all,dec_fc_out,4096^3"
step() { timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-also | cut -c1-140; }
case "${1:-stage}" in
  stage) for r in 1 2; do for a in 0 1 2; do echo "## stage $a"; MIT_G256_STAGE=$a GEMM_SHAPES=$SH timeout -k 10 100 python -u tools/gemm_bench.py 2 || exit 1; done; done
         for a in 0 1 2 0 1 2; do echo "## stage $a $(MIT_G256_STAGE=$a step)"; done ;;
  persist) for r in 1 2; do for a in 0 8; do echo "## variant $a"; MIT_G256_PERSIST=1 GEMM_SHAPES=$SH timeout -k 10 100 python -u tools/gemm_bench.py $a || exit 1; done; done
           for a in 1 0 1 0; do echo "## persist $a $(MIT_G256_PERSIST=$a step)"; done ;;
  tall) GEMM_SHAPES=$SH timeout -k 10 200 python -u tools/gemm_bench.py 2,7 ;;
  grouped) for a in 8 1 8 1; do echo "## group $a $(MIT_GROUPED_GROUP=$a step)"; done ;;
  nowait) for l in multimodal-image-transformer_amd/lib/libmit_hip.so $V/libmit_hip_nowait.so; do echo "## $l"; MIT_LIB=$l GEMM_SHAPES=$SH timeout -k 10 100 python -u tools/gemm_bench.py 2 || exit 1; done ;;
  stamps) MIT_LIB=$V/libmit_hip_stamp.so timeout -k 10 150 python -u tools/g256_stamps.py iso8 iso8_res enc_qkv+bias enc_o+res enc_fc1+gelu enc_fc2+res ;;
esac
