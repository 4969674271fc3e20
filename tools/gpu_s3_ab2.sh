# Session-3 A/B (interleaved, one box): stream priorities (MIT_STREAM_PRIORITY) and the grouped dW
# split-K factor (MIT_GROUPED_SPLIT, 0 = per-group default = 2 at cfg1)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_ab2
mkdir -p $OUT
run() { # name, env...
  n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > $OUT/$n.json 2> $OUT/$n.err || exit 1
  echo "$n $(python3 -c "import json;d=json.load(open('$OUT/$n.json'));print(d['value'], d['ms_per_step'])")"
}
for r in 1 2; do
  run base.$r MIT_STREAM_PRIORITY=0
  run prio.$r MIT_STREAM_PRIORITY=1
  run gs1.$r MIT_GROUPED_SPLIT=1
  run gs3.$r MIT_GROUPED_SPLIT=3
  run gs4.$r MIT_GROUPED_SPLIT=4
  run nogroup.$r MIT_DW_GROUPED=0
done
