# attention tests on the lazy-rescale build, then attn_bench and the step, lazy vs rescale-every-chunk
# (lib/libmit_hip_nolazy.so: attention.hip built with -DMIT_ATTN_LAZY=0; the lazy build: -DMIT_ATTN_LAZY=8),
# interleaved; LAZY_TESTS=1 runs the parity tests first
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NL=/root/repo/multimodal-image-transformer_amd/lib/libmit_hip_nolazy.so
[ -n "$LAZY_TESTS" ] && { timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_bf16_parity_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/tlazy.log 2>&1; rc=$?; tail -2 gpurun_out/tlazy.log; [ $rc -eq 0 ] || exit $rc; }
for r in 1 2; do
  echo "[nolazy] r$r"; MIT_HIP_LIB=$NL timeout -k 10 120 python -u tools/attn_bench.py || exit 1
  echo "[lazy] r$r"; timeout -k 10 120 python -u tools/attn_bench.py || exit 1
done
bash tools/gpu_ab.sh -r 3 "MIT_HIP_LIB=$NL" "MIT_LAZY=1"
