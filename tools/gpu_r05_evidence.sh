# round-5 measurement evidence on the current tree: an un-profiled default bench line, the rocprofv3 passes of
# tools/profile_round.sh (trace, no-prefetch trace, FETCH_SIZE, WRITE_SIZE, MFMA-busy; condensed), and the
# long-dispatch clock pass (tools/clock_pass.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py > gpurun_out/bench_r05.json 2> gpurun_out/bench_r05.err || { tail -20 gpurun_out/bench_r05.err; exit 1; }
cut -c1-400 gpurun_out/bench_r05.json
bash tools/profile_round.sh r05 || exit 1
cat gpurun_out/prof_r05/keep/summary.txt
bash tools/clock_pass.sh || exit 1
cp gpurun_out/clock_pass.json gpurun_out/prof_r05/keep/r05_clock_pass.json
