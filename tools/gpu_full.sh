# full GPU test suite + default bench (gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
