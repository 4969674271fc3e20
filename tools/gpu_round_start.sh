# Baseline of the current tree on a fresh box: the default bench line, then tools/profile_round.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/start
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && cut -c1-400 $OUT/bench.json &&
bash tools/profile_round.sh ${1:-r04}
