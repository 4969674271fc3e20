# A/B of run-time knobs on the default bench (interleaved, one box): each line = one bench run
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for round in 1 2; do
  for v in "base" "MIT_GEMM_FUSED_SPLIT=1" "MIT_DW_SIDE_STREAM=0" "NOPF"; do
    if [ "$v" = "base" ]; then e=""; a=""; elif [ "$v" = "NOPF" ]; then e=""; a="--no-prefetch"; else e="$v"; a=""; fi
    r=$(env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $a 2>/dev/null) || { echo "$v failed"; exit 1; }
    echo "$round $v $(echo $r | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
  done
done
