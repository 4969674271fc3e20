#!/bin/bash
# SQ stall split of the encoder's 256-tile GEMM shapes (tools/gemm_bench.py, one shape set, bf16): two
# --pmc passes of their own (8 SQ + 1 GRBM counters, then 8 SQ), each under its own time limit, condensed
# by tools/sq_split.py into gpurun_out/sq/<TAG>_sq_split.json. Usage: bash tools/gemm_sq_split.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06}
O=gpurun_out/sq
mkdir -p $O
export GEMM_SHAPES=${GEMM_SHAPES:-"enc fc1+gelu+ln,enc fc1,enc o+res+st,enc fc2+res+st,enc qkv+ln,4096^3"}
P="rocprofv3 --output-format csv"
timeout -s KILL 120 $P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $O/a -o run -- python3 tools/gemm_bench.py ${GEMM_VARIANTS:-2n} > $O/a.log 2>&1 &&
timeout -s KILL 120 $P --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  -d $O/b -o run -- python3 tools/gemm_bench.py ${GEMM_VARIANTS:-2n} > $O/b.log 2>&1 &&
python3 tools/sq_split.py $(find $O/a -name '*counter_collection.csv' | head -n 1) --json $O/${TAG}_sq_split_a.json > $O/${TAG}_sq_a.txt &&
python3 tools/sq_split.py $(find $O/b -name '*counter_collection.csv' | head -n 1) --json $O/${TAG}_sq_split_b.json > $O/${TAG}_sq_b.txt &&
rm -rf $O/a $O/b
