cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t256.log 2>&1; rc=$?; tail -3 gpurun_out/t256.log; [ $rc -eq 0 ] || exit $rc
GEMM_SHAPES="enc o,enc fc2+res,enc fc2,enc qkv+bias,enc fc1+gelu,clip o+res,clip fc2+res,clip qkv,clip fc1+gelu,cfg3 o+res,cfg3 fc2+res" timeout -k 10 300 python -u tools/gemm_bench.py 2,6,5
