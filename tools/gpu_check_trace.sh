# full GPU tests, default bench, and a no-prefetch kernel trace (per-kernel step breakdown)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench.json 2>/dev/null &&
rm -rf gpurun_out/tr_np && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_np -o run -- python3 bench.py --no-cpu-baseline --no-roofline --no-prefetch --steps 6 --warmup 2 > gpurun_out/tr_np.json 2>/dev/null
