# L2 hit rate of the GEMM kernels on train-step shapes (gemm_bench), one TCC pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gemm_pmc
GEMM_SHAPES="enc fc1,enc qkv,enc fc2,dX lin1+res,fwd out+bias" timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/gemm_pmc/p1 -o run -- python3 tools/gemm_bench.py 0 > gpurun_out/gemm_pmc/p1.txt 2>&1
