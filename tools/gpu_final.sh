# full GPU suite + smoke + default bench + rocprofv3 kernel stats of the configs[2] workload (gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_clip336 -o run -- python3 bench.py --workload clip336 --steps 5 --warmup 2 --no-roofline > gpurun_out/prof_clip336.log 2>&1
