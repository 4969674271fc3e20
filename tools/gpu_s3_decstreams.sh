# Session-3: decode tests, then the configs[4] line per row-group count (MIT_DECODE_STREAMS) with the
# native plan replay (default) and with per-group hipGraphs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_decstreams${MIT_TAG}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py > $OUT/pytest.log 2>&1 &&
tail -2 $OUT/pytest.log || exit 1
for g in 1 2 3 4; do
  MIT_DECODE_STREAMS=$g timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/plan_g$g.json 2> $OUT/plan_g$g.err || exit 1
  echo "plan G=$g $(python3 -c "import json;d=json.load(open('$OUT/plan_g$g.json'));print(d['value'], d['us_per_token_step'])")"
done
MIT_DECODE_STREAMS=1 MIT_DECODE_LAUNCH=graph timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/graph_g1.json 2> $OUT/graph_g1.err || exit 1
echo "graph G=1 $(python3 -c "import json;d=json.load(open('$OUT/graph_g1.json'));print(d['value'], d['us_per_token_step'])")"
