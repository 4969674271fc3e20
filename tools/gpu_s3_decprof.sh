# Session-3: rocprofv3 kernel stats of the configs[4] decode (fused bf16 step)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s3_decprof${MIT_TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --workload decode --no-cpu-baseline --steps 2 --warmup 1 > $OUT/trace.json 2> $OUT/trace.err
