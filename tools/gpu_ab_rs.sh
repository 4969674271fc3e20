# 64x64 register-streaming NT GEMM (MIT_GEMM_RS=1 / variant 3): parity tests, per-shape times with it
# on and off, the train bench and the decode bench with it on and off
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/rs
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
MIT_GEMM_RS=1 timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_model.log 2>&1
rc=$?; tail -3 $OUT/pytest_model.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas_0.txt 2>&1 || exit 1
MIT_GEMM_RS=1 timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas_1.txt 2>&1 || exit 1
paste -d'|' $OUT/blas_0.txt $OUT/blas_1.txt | cut -c1-62,95-140
for r in 1 2; do for v in 0 1; do
  echo "$r train rs=$v $(MIT_GEMM_RS=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
for v in 0 1; do
  echo "decode rs=$v $(MIT_GEMM_RS=$v timeout -k 10 200 python bench.py --workload decode --no-cpu-baseline --no-roofline 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("ms_per_step"))')"
done
