# A/B of an env knob on the default bench, interleaved (gpurun from the repo root): bash tools/gpu_ab.sh VAR
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=${1:-MIT_GEMM_FUSED_SPLIT}
for r in 1 2; do
  env $V=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/ab_on_$r.json 2>/dev/null &&
  env $V=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/ab_off_$r.json 2>/dev/null || exit 1
done
