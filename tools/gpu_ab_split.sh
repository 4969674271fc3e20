# split-K block target for the plain-epilogue weight-gradient GEMMs (MIT_SPLITK_TARGET), bench A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in 128 64 16; do
  echo "$r target=$v $(MIT_SPLITK_TARGET=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
