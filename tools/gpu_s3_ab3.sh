# Session-3 A/B (interleaved, one box): in-launch split-K combine for the long-K data gradients
# (MIT_GEMM_FUSED_MINK: 0 = off, 1536 = linear1 + self in_proj dX, 2048 = linear1 dX only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_ab3
mkdir -p $OUT
run() { # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/$n.json 2> $OUT/$n.err || exit 1
  echo "$n $(python3 -c "import json;d=json.load(open('$OUT/$n.json'));print(d['value'], d['ms_per_step'])")"
}
for r in 1 2 3; do
  run k0.$r MIT_GEMM_FUSED_MINK=0
  run k1536.$r MIT_GEMM_FUSED_MINK=1536
  run k2048.$r MIT_GEMM_FUSED_MINK=2048
done
