# r04i: LN-fold statistics merged once per tile row in the prologue: GEMM/encoder tests, then the step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04i
timeout -k 10 400 python -u -m pytest tests/test_gemm256_gpu.py tests/test_model_gpu.py tests/test_bf16_parity_gpu.py tests/test_asserts_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/r04i/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04i/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-also --steps 30 --warmup 5"
for r in 1 2 3; do
  echo "## new $(timeout -k 10 120 python -u bench.py $B | cut -c90-130)"
done
timeout -k 10 200 python -u tools/step_parts.py || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04i/prof -o run -- python3 bench.py --no-cpu-baseline --no-also --no-roofline --steps 10 --warmup 3 > gpurun_out/r04i/prof.log 2>&1 || exit 1
