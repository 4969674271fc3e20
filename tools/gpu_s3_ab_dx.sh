# Session-3: decode tests + decode bench (fused step), then an interleaved train-step A/B of the
# split-K block target for the K-contig-A (data-gradient) GEMMs (MIT_SPLITK_TARGET_DX).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_ab${MIT_TAG}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py > $OUT/pytest.log 2>&1 &&
tail -3 $OUT/pytest.log &&
timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/decode.json 2> $OUT/decode.err &&
cat $OUT/decode.json &&
for r in 1 2; do
  for t in 128 256 512; do
    MIT_SPLITK_TARGET_DX=$t timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/train_dx$t.$r.json 2> $OUT/train_dx$t.$r.err || exit 1
    echo "dx$t r$r $(python3 -c "import json;d=json.load(open('$OUT/train_dx$t.$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
