# r04k: bias / column sums staged into LDS in the 256 kernel's prologue: GEMM tests + same-box A/B vs HEAD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04k
timeout -k 10 400 python -u -m pytest tests/test_gemm256_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_asserts_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/r04k/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04k/tests.log; [ $rc -eq 0 ] || exit $rc
V=multimodal-image-transformer_amd/lib/ab/libmit_hip_head.so
B="--no-cpu-baseline --no-also --steps 30 --warmup 5"
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d.get("roofline") or {}; print(d["value"], r.get("avg_launch_us"))'
for r in 1 2 3; do
  echo "## new $(timeout -k 10 120 python -u bench.py $B | python3 -c "$S")"
  echo "## head $(MIT_LIB=$V timeout -k 10 120 python -u bench.py $B | python3 -c "$S")"
done
