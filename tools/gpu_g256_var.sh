# GEMM-256 schedule variants: parity/race tests, microbench, interleaved default benches
# usage (gpurun from the repo root): bash tools/gpu_g256_var.sh VARIANT...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=multimodal-image-transformer_amd/lib
for v in "$@"; do
  MIT_LIB=$L/variants/libmit_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py -m gpu > gpurun_out/g256t_$v.log 2>&1 || exit 1
done
bash tools/gpu_g256_ab.sh "$@"
