# Round-2 bench pass: the default bench line (replay path, CPU baseline), the eager launch path for
# comparison, the per-shape GEMM comparison against hipBLASLt, and a kernel trace of the step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/bench_r02${MIT_TAG}
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --no-replay > $OUT/bench_eager.json 2> $OUT/bench_eager.err &&
cat $OUT/bench_eager.json &&
timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas.txt 2>&1 &&
cat $OUT/blas.txt &&
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-roofline --steps 10 --warmup 3 > $OUT/trace.json 2> $OUT/trace.err
