# interleaved A/B/C of an env knob's values on the default bench: bash tools/gpu_ab3.sh VAR v1 v2 v3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=$1; shift
for r in 1 2; do
  for val in "$@"; do
    env $V=$val timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/ab3_${val}_$r.json 2>/dev/null || exit 1
  done
done
