# head-resident vs 64-query-block attention forward on the train workloads: bash tools/gpu_attn_ab.sh WORKLOAD...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for w in "$@"; do
    for hv in 1 0; do
      MIT_ATTN_HEAD=$hv timeout -k 10 200 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/attn_ab_${w}_${hv}_$r.json 2>/dev/null || exit 1
    done
  done
done
