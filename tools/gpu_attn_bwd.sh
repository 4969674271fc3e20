set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/attn_bwd
timeout -k 10 120 python -u tools/attn_bwd_bench.py > gpurun_out/attn_bwd/bench.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/attn_bwd/prof -o run -- python3 tools/attn_bwd_bench.py > gpurun_out/attn_bwd/prof.txt 2>&1
