# Gathered GEMM epilogues: GEMM + model parity tests, per-shape times vs hipBLASLt, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/epi${MIT_TAG}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gemm256_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas.txt 2>&1 && cat $OUT/blas.txt &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json
