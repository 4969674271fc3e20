# r04h: decoder work on CU-masked streams (bench --decoder-cus), same-box A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u -m pytest tests/test_plan_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r04h/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04h/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-also --no-roofline --steps 30 --warmup 5"
for r in 1 2; do
  echo "## none $(timeout -k 10 120 python -u bench.py $B | cut -c90-130)"
  for m in 64/4 96 128/2 64 32/8 160 ~64; do
    echo "## $m $(timeout -k 10 120 python -u bench.py $B --decoder-cus $m | cut -c90-130)"
  done
done
