# 8-wave 128x128 kernel (MIT_GEMM_W8: 1 = grids of <= one block per CU, 2 = always) vs the 4-wave one:
# GEMM parity under each mode, per-shape times, train bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/w8
mkdir -p $OUT
for v in 1 2; do
MIT_GEMM_W8=$v timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1
rc=$?; tail -2 $OUT/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in 0 1 2; do MIT_GEMM_W8=$v timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas_$v.txt 2>&1 || exit 1; done
paste -d'|' $OUT/blas_0.txt $OUT/blas_1.txt $OUT/blas_2.txt | cut -c1-62,95-142,175-222
for r in 1 2; do for v in 0 1 2; do
  echo "$r w8=$v $(MIT_GEMM_W8=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
