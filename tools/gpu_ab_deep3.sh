# 3 LDS stages for the 8-wave 128 kernel on <= 1-block-per-CU grids (MIT_GEMM_DEEP3=1) vs 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/deep3
mkdir -p $OUT
MIT_GEMM_DEEP3=1 timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do MIT_GEMM_DEEP3=$v timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas_$v.txt 2>&1 || exit 1; done
paste -d'|' $OUT/blas_0.txt $OUT/blas_1.txt | cut -c1-62,95-142
for r in 1 2; do for v in 0 1; do
  echo "$r deep3=$v $(MIT_GEMM_DEEP3=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
