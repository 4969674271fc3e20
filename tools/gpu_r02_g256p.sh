# Persistent 256 GEMM: parity tests, isolated A/B, then the bench with it on and off
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/g256p${MIT_TAG}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm256p_ab.py > $OUT/ab.txt 2>&1 && cat $OUT/ab.txt &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/bench_p1.json 2> $OUT/bench_p1.err && cat $OUT/bench_p1.json &&
MIT_G256P=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/bench_p0.json 2> $OUT/bench_p0.err && cat $OUT/bench_p0.json
