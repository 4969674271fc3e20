# One GPU call for a build: the -m gpu suite, then (only if it is green) the default bench line and the
# rocprofv3 passes of tools/profile_round.sh. Usage: bash tools/gpu_round.sh TAG [skip-tests]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -25 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc: no bench"; exit $rc; }
fi
timeout -k 10 420 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
cut -c1-600 gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
bash tools/profile_round.sh $TAG
