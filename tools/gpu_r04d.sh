# r04d: encoder-prefetch interleave A/B (MIT_AB_ENC_LEAD chunks before the decoder; 99 = all up front)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04d
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_plan_gpu.py tests/test_bench_gate_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/r04d/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04d/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-also --no-roofline --steps 30 --warmup 5"
for r in 1 2; do
  for v in 99 0 1 2 4; do
    echo "## lead $v $(MIT_AB_ENC_LEAD=$v timeout -k 10 200 python -u bench.py $B | cut -c90-150)"
  done
done
