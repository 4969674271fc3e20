# SQ counters of the 128 kernel (8 waves) on the d_model = 512 decoder shapes (gemm_bench, variant 1):
# wave-cycle split (issuing / waiting / idle), MFMA busy, LDS bank conflicts; one pass per counter set
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/gemm128_sq
mkdir -p $OUT
export GEMM_SHAPES="fwd out+bias,fwd lin2+res,dX lin1+res,dX out"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o run -- python3 tools/gemm_bench.py 1 > $OUT/p1.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES --output-format csv -d $OUT/p2 -o run -- python3 tools/gemm_bench.py 1 > $OUT/p2.txt 2>&1
rc=$?; cat $OUT/p1.txt; exit $rc
