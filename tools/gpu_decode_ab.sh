# (historical, round 1) tiny-grid split-K in the decode token step — the MIT_GEMM_TINY_SPLIT switch it
# toggled was reverted after this A/B (profiles/r01_decode_profile.txt); kept as the recipe of that measurement
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py tests/test_gemm256_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/decode_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 1 0; do
    MIT_GEMM_TINY_SPLIT=$v timeout -k 10 200 python -u bench.py --workload decode > gpurun_out/dec_ab_${v}_$r.json 2>/dev/null || exit 1
  done
done
