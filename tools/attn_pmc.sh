set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 && MIT_ATTN_HEAD=0 python tools/attn_bench.py >> gpurun_out/attn_bench.log 2>&1 || exit 1
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/attn_pmc$i -o run -- python3 tools/attn_bench.py > /dev/null 2>&1 || exit 1
done
