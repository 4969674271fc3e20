# Session-3: decode tests, configs[4] line with the long-K 8-wave decode GEMM and the per-image decode
# attention on / off, kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_decab${MIT_TAG}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py > $OUT/pytest.log 2>&1 &&
tail -2 $OUT/pytest.log || exit 1
for r in 1 2; do
for v in "1 1" "0 1" "1 0"; do
  set -- $v
  MIT_DECODE_LONGK=$1 MIT_DECODE_ROWS_ATTN=$2 timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/l$1a$2.$r.json 2> $OUT/l$1a$2.$r.err || exit 1
  echo "longk=$1 rows_attn=$2 $(python3 -c "import json;d=json.load(open('$OUT/l$1a$2.$r.json'));print(d['value'], d['us_per_token_step'])")"
done
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --workload decode --no-cpu-baseline --steps 2 --warmup 1 > $OUT/trace.json 2> $OUT/trace.err
