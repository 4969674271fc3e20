# interleaved A/B of the head-resident attention's staging knobs (tools/attn_bench.py, one process each)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in "MIT_ATTN_PAD=64" "MIT_ATTN_PAD=16"; do
    echo "[$v] r$r"; env $v timeout -k 10 120 python -u tools/attn_bench.py || exit 1
  done
done
