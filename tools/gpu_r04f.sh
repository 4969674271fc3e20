# r04f: split-K with bias / residual for the decoder's long-K GEMMs: tests + same-box A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_bf16_parity_gpu.py tests/test_decode_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/r04f/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04f/tests.log; [ $rc -eq 0 ] || exit $rc
V=multimodal-image-transformer_amd/lib/ab/libmit_hip_nosplitepi.so
B="--no-cpu-baseline --no-also --steps 30 --warmup 5"
for r in 1 2 3; do
  echo "## split $(timeout -k 10 200 python -u bench.py $B | cut -c90-150)"
  echo "## nosplit $(MIT_LIB=$V timeout -k 10 200 python -u bench.py $B | cut -c90-150)"
done
timeout -k 10 200 python -u bench.py $B > gpurun_out/r04f/bench.json 2>&1
timeout -k 10 200 python -u tools/step_parts.py
MIT_LIB=$V timeout -k 10 200 python -u tools/step_parts.py
