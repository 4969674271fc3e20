# Session-3: GELU epilogue A/B (A&S 7.1.26 default vs 7.1.28 variant lib): per-shape GEMM times, the
# train step, and the GELU parity tests under the variant
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_gelu
mkdir -p $OUT
V=$GRAFT_REPO_ROOT/multimodal-image-transformer_amd/lib/variants/libmit_hip_as28.so
MIT_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gelu or GELU or act" > $OUT/pytest_as28.log 2>&1; tail -2 $OUT/pytest_as28.log
timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas_default.txt 2>&1 &&
MIT_LIB=$V timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas_as28.txt 2>&1 &&
grep -E 'fc1|sum' $OUT/blas_default.txt $OUT/blas_as28.txt || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/train_def.$r.json 2>/dev/null || exit 1
  MIT_LIB=$V timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/train_as28.$r.json 2>/dev/null || exit 1
  echo "r$r default $(python3 -c "import json;print(json.load(open('$OUT/train_def.$r.json'))['value'])") as28 $(python3 -c "import json;print(json.load(open('$OUT/train_as28.$r.json'))['value'])")"
done
