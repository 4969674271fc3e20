#!/bin/bash
# Interleaved A/B of run-time knobs on ONE box (box-to-box spread is ~3 %, so only same-box,
# interleaved rounds are compared):
#   tools/gpu_ab.sh [-w WORKLOAD] [-r ROUNDS] "KNOB=a [KNOB2=b]" "KNOB=c" ...
# Each variant is one bench.py run (--no-cpu-baseline --no-roofline) with those environment
# assignments; prints "variant round value ms_per_step". The session-3 numbers in DESIGN §4.1c / §5.1
# were taken this way, e.g. MIT_DW_GROUPED=1 / 0, MIT_GROUPED_SPLIT=1..4, MIT_STREAM_PRIORITY=0 / 1,
# MIT_SPLITK_TARGET_DX=128 / 256 / 512, MIT_GEMM_FUSED_MINK=0 / 1536 / 2048, and for -w decode
# MIT_DECODE_FUSED, MIT_DECODE_LONGK, MIT_DECODE_ROWS_ATTN, MIT_DECODE_STREAMS, MIT_DECODE_LAUNCH.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=train; R=2
while getopts "w:r:" o; do case $o in w) W=$OPTARG ;; r) R=$OPTARG ;; *) exit 2 ;; esac; done
shift $((OPTIND - 1))
OUT=gpurun_out/ab_$W
mkdir -p $OUT
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    env $v timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --no-roofline > $OUT/v$i.$r.json 2> $OUT/v$i.$r.err || exit 1
    echo "[$v] r$r $(python3 -c "import json;d=json.load(open('$OUT/v$i.$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
