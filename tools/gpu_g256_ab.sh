# GEMM-256 tile-order variants (tools/build_variants.sh): microbench on the 256-tile shapes, then
# interleaved default benches (gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=multimodal-image-transformer_amd/lib
export GEMM_SHAPES="enc qkv,enc o,enc fc1+gelu,enc fc2+res,dec kv_all,dec fc_out"
for v in base "$@"; do
  lib=$L/libmit_hip.so; [ $v != base ] && lib=$L/variants/libmit_hip_$v.so
  MIT_LIB=$lib timeout -k 10 120 python -u tools/gemm_bench.py 2 > gpurun_out/g256_$v.txt 2>&1 || exit 1
done
for r in 1 2; do
  for v in base "$@"; do
    lib=$L/libmit_hip.so; [ $v != base ] && lib=$L/variants/libmit_hip_$v.so
    MIT_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/g256b_${v}_$r.json 2>/dev/null || exit 1
  done
done
