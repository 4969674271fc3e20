# Session-3 decode pass: decode tests, the configs[4] bench line (fused step, then the 12-launch step
# for comparison), and a rocprofv3 kernel summary of the fused step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_decode${MIT_TAG}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_decode_gpu.py > $OUT/pytest.log 2>&1 &&
tail -3 $OUT/pytest.log &&
timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
MIT_DECODE_FUSED=0 timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/bench_unfused.json 2> $OUT/bench_unfused.err &&
cat $OUT/bench_unfused.json &&
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --workload decode --no-cpu-baseline --steps 2 --warmup 1 > $OUT/trace.json 2> $OUT/trace.err
