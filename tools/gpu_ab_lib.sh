# A/B of a compile-time kernel variant (tools/build_variants.sh -> lib/ab/libmit_hip_NAME.so) against the
# default build on one box: the -m gpu tests matching PYTEST_K under the variant, then MICRO (a tools/ micro
# benchmark, with its ARGS) and the train step (bench.py, no CPU baseline / also / roofline), interleaved.
#   bash tools/gpu_ab_lib.sh NAME "PYTEST_K" MICRO "MICRO_ARGS" [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=multimodal-image-transformer_amd/lib/ab/libmit_hip_$1.so
R=${5:-2}
mkdir -p gpurun_out
MIT_LIB=$V timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "$2" --timeout 120 --timeout-method thread \
  > gpurun_out/ab_$1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_$1_tests.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq 1 $R); do
  echo "## default $3"; timeout -k 10 200 python -u tools/$3 $4 || exit 1
  echo "## $1 $3"; MIT_LIB=$V timeout -k 10 200 python -u tools/$3 $4 || exit 1
done
B="--no-cpu-baseline --no-also --no-roofline --steps 20 --warmup 5"
for r in $(seq 1 $R); do
  echo "## default step $(timeout -k 10 200 python -u bench.py $B | cut -c1-140)"
  echo "## $1 step $(MIT_LIB=$V timeout -k 10 200 python -u bench.py $B | cut -c1-140)"
done
