# Session-3: embedding-gradient row batching -- embedding / train-step parity tests, then the train line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_emb
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "embed or train or prefetch or resume" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/t.$r.json 2> $OUT/t.$r.err || exit 1
  echo "r$r $(python3 -c "import json;d=json.load(open('$OUT/t.$r.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-roofline --steps 5 --warmup 2 > $OUT/trace.json 2> $OUT/trace.err
