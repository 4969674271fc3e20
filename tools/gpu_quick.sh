# GPU tests + attention bwd microbench + default bench (gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
true && timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
mkdir -p gpurun_out/attn_bwd && timeout -k 10 120 python -u tools/attn_bwd_bench.py > gpurun_out/attn_bwd/bench.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench.json 2> gpurun_out/bench.err
