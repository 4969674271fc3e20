# SQ counters of the 256 GEMM on the encoder shapes (gemm_bench, forced 256 tiles): stall breakdown and
# LDS bank conflicts, one pass (gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gemm_sq
GEMM_SHAPES="enc qkv,enc o,enc fc2+res" timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/gemm_sq/p1 -o run -- python3 tools/gemm_bench.py 2 > gpurun_out/gemm_sq/p1.txt 2>&1
