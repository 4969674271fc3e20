#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root; outputs to gpurun_out/):
#   1) kernel trace + stats of the default bench command (native replay, encoder prefetch stream,
#      weight-gradient side stream) -> trace   [timeline: tools/timeline.py]
#   2) the same with --no-prefetch (encoder inline: per-kernel attribution without overlap)
#   3) FETCH_SIZE and 4) WRITE_SIZE, each in its own pass (TCC slots; MI355X_MICROARCH.md HBM
#      section) over the default command
#   5) MFMA-busy + clock: SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE in one
#      pass of their own (3 SQ + 1 GRBM counters, within one pass's limits)
# Condensed at the end (tools/rocpd_summary.py, tools/step_timeline.py) into $OUT/keep -> profiles/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# WORKLOAD=clip336 / cfg3: the same passes over that workload (bench.py --workload)
ARGS="--no-cpu-baseline --no-also --steps 10 --warmup 3${WORKLOAD:+ --workload $WORKLOAD}"
P="rocprofv3 --output-format rocpd csv"
timeout -k 10 300 $P --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.json 2> $OUT/trace.err &&
timeout -k 10 300 $P --kernel-trace --stats -d $OUT/trace_noprefetch -o run -- python3 bench.py $ARGS --no-prefetch --no-roofline > $OUT/trace_noprefetch.json 2> $OUT/trace_noprefetch.err &&
timeout -k 10 300 $P --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run -- python3 bench.py $ARGS --no-roofline > $OUT/fetch.json 2> $OUT/fetch.err &&
timeout -k 10 300 $P --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run -- python3 bench.py $ARGS --no-roofline > $OUT/write.json 2> $OUT/write.err &&
timeout -s KILL 300 $P --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq -o run -- python3 bench.py $ARGS --no-roofline > $OUT/sq.json 2> $OUT/sq.err
# condense on the box (the rocpd databases exceed gpurun_out's copy-back cap): summaries under
# $OUT/keep, databases deleted
f() { find $OUT/$1 -name "$2" | head -n 1; }
mkdir -p $OUT/keep &&
python3 tools/rocpd_summary.py --trace $(f trace '*results.db') --fetch $(f fetch '*results.db') \
  --write $(f write '*results.db') --sq $(f sq '*results.db') --trace-csv $(f trace '*kernel_trace.csv') --bench-json $OUT/trace.json $( [ -f gpurun_out/bench_$TAG.json ] && echo --bench-plain gpurun_out/bench_$TAG.json ) \
  --command "rocprofv3 --kernel-trace --stats / --pmc FETCH_SIZE / --pmc WRITE_SIZE / --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -- python3 bench.py $ARGS" \
  --out $OUT/keep/$TAG > $OUT/keep/summary.txt &&
cp $(f trace '*kernel_stats.csv') $OUT/keep/${TAG}_bench_kernel_stats.csv &&
cp $(f trace_noprefetch '*kernel_stats.csv') $OUT/keep/${TAG}_bench_noprefetch_kernel_stats.csv &&
python3 tools/step_timeline.py $(f trace '*kernel_trace.csv') > $OUT/keep/${TAG}_step_breakdown.txt &&
python3 tools/step_timeline.py $(f trace_noprefetch '*kernel_trace.csv') > $OUT/keep/${TAG}_step_breakdown_noprefetch.txt &&
rm -rf $OUT/trace $OUT/trace_noprefetch $OUT/fetch $OUT/write $OUT/sq
