# GEMM kernel checks + decoder-shape microbench (gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm256_gpu.py tests/test_kernels_gpu.py -k "gemm" > gpurun_out/g128_tests.log 2>&1 &&
GEMM_SHAPES="fwd out+bias,fwd lin2+res,dX out,dX q+res,dX lin1+res,dX self_in+res,dX fc_out ws,dW dd ws,dW ffn ws,dec ffn1" timeout -k 10 300 python -u tools/gemm_bench.py 0,0n,3 > gpurun_out/gemm_bench7.log 2>&1
