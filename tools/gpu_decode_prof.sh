#!/bin/bash
# configs[4] kernel stats under rocprofv3 (tools/, GPU box): one warmup call + one timed call of
# bench.py --workload decode, with and without the next call's encoder beside the token steps
set -e
OUT=${1:-gpurun_out/decprof}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/np" -o dec -- \
  python3 "$ROOT/bench.py" --workload decode --no-cpu-baseline --no-roofline --steps 4 --warmup 2 --no-prefetch \
  > "$ROOT/$OUT/np.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/pf" -o dec -- \
  python3 "$ROOT/bench.py" --workload decode --no-cpu-baseline --no-roofline --steps 4 --warmup 2 \
  > "$ROOT/$OUT/pf.log" 2>&1
echo done
