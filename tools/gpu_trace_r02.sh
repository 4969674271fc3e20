# Kernel trace of the default bench step (tools/step_timeline.py, tools/trace_step.py read it)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/trace_r02${MIT_TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $OUT -o run -- python3 bench.py --no-cpu-baseline --no-roofline --steps 10 --warmup 3 ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?
cat $OUT/bench.json
find $OUT -name "*kernel_trace.csv" | head -3
exit $rc
