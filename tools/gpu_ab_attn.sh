# A/B of the encoder attention forward: default build vs lib/ab/libmit_hip_$1.so (tools/build_variants.sh):
# the attention kernel tests under the variant, then tools/attn_bench.py interleaved (3 rounds)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=multimodal-image-transformer_amd/lib/ab/libmit_hip_$1.so
mkdir -p gpurun_out
MIT_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -q -k "attention or encoder" \
  --timeout 120 --timeout-method thread > gpurun_out/ab_attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_attn_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo "## default"; timeout -k 10 120 python -u tools/attn_bench.py || exit 1
  echo "## $1"; MIT_LIB=$V timeout -k 10 120 python -u tools/attn_bench.py || exit 1
done
