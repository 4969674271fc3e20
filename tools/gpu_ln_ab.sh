# LayerNorm forward tests + interleaved micro-benchmark of the row-per-wave variants (tools/ln_bench.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k layernorm --timeout 120 --timeout-method thread > gpurun_out/tln.log 2>&1; rc=$?; tail -2 gpurun_out/tln.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "MIT_LN_WIDE=0" "MIT_LN_RW=1" "MIT_LN_RW=2"; do
    echo "[$v] r$r"; env $v timeout -k 10 120 python -u tools/ln_bench.py || exit 1
  done
done
