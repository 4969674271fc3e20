# Refresh on the current build: the bench lines of every BASELINE workload, then the
# rocprofv3 kernel trace + FETCH/WRITE passes (tools/profile_round.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/refresh
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && cut -c1-300 $OUT/bench.json &&
timeout -k 10 300 python -u bench.py --workload decode --no-cpu-baseline > $OUT/decode.json 2> $OUT/decode.err && cut -c1-300 $OUT/decode.json &&
timeout -k 10 300 python -u bench.py --workload clip336 --no-cpu-baseline --steps 10 > $OUT/clip336.json 2> $OUT/clip336.err && cut -c1-300 $OUT/clip336.json &&
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --steps 10 > $OUT/cfg3.json 2> $OUT/cfg3.err && cut -c1-300 $OUT/cfg3.json &&
bash tools/profile_round.sh
