cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
timeout -k 10 300 python -u tools/blas_reference.py > $OUT/blas.txt 2>&1 &&
cat $OUT/blas.txt
