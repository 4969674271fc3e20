# Round-2 refresh on the current build: full bench line (default flags, CPU baseline), the other
# BASELINE workloads, a fused-split-K A/B, then rocprofv3 kernel trace + FETCH/WRITE passes
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/refresh
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json | cut -c1-400 &&
timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/decode.json 2> $OUT/decode.err && cut -c1-300 $OUT/decode.json &&
timeout -k 10 300 python -u bench.py --workload clip336 --no-cpu-baseline --steps 10 > $OUT/clip336.json 2> $OUT/clip336.err && cut -c1-300 $OUT/clip336.json &&
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --steps 10 > $OUT/cfg3.json 2> $OUT/cfg3.err && cut -c1-300 $OUT/cfg3.json || exit 1
for r in 1 2; do for v in 0 1; do
  echo "$r fused=$v $(MIT_GEMM_FUSED_SPLIT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
bash tools/profile_r02.sh
