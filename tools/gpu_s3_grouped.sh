# Session-3: grouped per-layer dW -- kernel + train-step parity tests, then an interleaved train-step
# A/B (MIT_DW_GROUPED=1 vs 0) and the gemm class breakdown of the default line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_grouped
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_bf16_parity_gpu.py tests/test_model_gpu.py tests/test_dist_gpu.py tests/test_plan_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    MIT_DW_GROUPED=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/train_g$v.$r.json 2> $OUT/train_g$v.$r.err || exit 1
    echo "grouped=$v r$r $(python3 -c "import json;d=json.load(open('$OUT/train_g$v.$r.json'));print(d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])")"
  done
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], json.dumps(d['gemm_breakdown']))"
