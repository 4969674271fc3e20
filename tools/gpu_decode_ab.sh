# decode: parity tests on the current build, then the decode bench, plus a rocprofv3 kernel-stats pass
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/decode${MIT_TAG}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/decode.json 2> $OUT/decode.err && cut -c1-200 $OUT/decode.json &&
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --workload decode --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof.json 2> $OUT/prof.err
