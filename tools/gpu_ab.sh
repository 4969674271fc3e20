#!/bin/bash
# Interleaved A/B of run-time knobs on ONE box (box-to-box spread is ~3 %, so only same-box,
# interleaved rounds are compared):
#   tools/gpu_ab.sh [-k PYTEST_EXPR] [-m MICRO_BENCH] [-w WORKLOAD] [-r ROUNDS] "KNOB=a [KNOB2=b]" "KNOB=c" ...
# -k first runs the -m gpu tests matching PYTEST_EXPR ("all" = the whole suite) on the default build and
# stops if they fail. Each variant is then one run with those environment assignments, R interleaved
# rounds: of bench.py (--no-cpu-baseline --no-roofline; prints "variant round value ms_per_step"), or
# with -m of a kernel micro-benchmark (tools/gemm_bench.py, attn_bench.py, ln_bench.py; a variant
# "ARGS=..." passes its arguments, e.g. ARGS=2,6,5 for gemm_bench's tile variants). Variants may
# select a library build with MIT_HIP_LIB=<path> (tools/build_variants.sh builds one with compile-time
# flags); that is how kernel variants are compared (the round-1..3 run-time knobs of DESIGN §4.1c /
# §4.1d / §5.1 were measured this way and have since been folded into their measured defaults).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=train; R=2; K=; MB=
while getopts "k:m:w:r:" o; do
  case $o in k) K=$OPTARG ;; m) MB=$OPTARG ;; w) W=$OPTARG ;; r) R=$OPTARG ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
OUT=gpurun_out/ab_$W
mkdir -p $OUT
if [ -n "$K" ]; then
  SEL=(-k "$K"); [ "$K" = all ] && SEL=()
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x "${SEL[@]}" --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1
  rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    if [ -n "$MB" ]; then
      echo "[$v] r$r"
      args=$(echo "$v" | sed -n 's/.*ARGS=\([^ ]*\).*/\1/p')
      env $(echo "$v" | sed 's/ARGS=[^ ]*//') timeout -k 10 300 python -u tools/$MB $args || exit 1
      continue
    fi
    env $v timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --no-roofline > $OUT/v$i.$r.json 2> $OUT/v$i.$r.err || exit 1
    echo "[$v] r$r $(python3 -c "import json;d=json.load(open('$OUT/v$i.$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
