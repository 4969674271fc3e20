# r04j: same-box A/B of the LN-fold prologue merge (current) against HEAD's epilogue merge (lib/ab/libmit_hip_head.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04j
V=multimodal-image-transformer_amd/lib/ab/libmit_hip_head.so
B="--no-cpu-baseline --no-also --steps 30 --warmup 5"
S='import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d.get("roofline") or {}; print(d["value"], r.get("avg_launch_us"), json.dumps(d.get("gemm_breakdown"))[:400])'
for r in 1 2 3; do
  echo "## new $(timeout -k 10 120 python -u bench.py $B | python3 -c "$S")"
  echo "## head $(MIT_LIB=$V timeout -k 10 120 python -u bench.py $B | python3 -c "$S")"
done
