# default bench + variants given as extra args lines (gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/b_default.json 2>/dev/null &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --no-prefetch > gpurun_out/b_noprefetch.json 2>/dev/null &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --graph > gpurun_out/b_graph.json 2>/dev/null
