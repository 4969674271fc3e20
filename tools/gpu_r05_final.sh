# round-5 evidence on the final tree, in two gpurun calls (each under the 20-minute limit):
#   bash tools/gpu_r05_final.sh tests  -> the -m gpu suite and smoke()
#   bash tools/gpu_r05_final.sh bench  -> the bench line (roofline + cpu_baseline + also), the rocprofv3
#                                         passes (tools/profile_round.sh r05), the long-dispatch clock
#                                         pass, un-profiled step parts
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "$1" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread \
    > gpurun_out/r05_pytest_gpu.log 2>&1
  rc=$?
  tail -15 gpurun_out/r05_pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke.log 2>&1 || exit 1
  tail -2 gpurun_out/r05_smoke.log
  exit 0
fi
bash tools/gpu_round.sh r05 skip-tests || exit 1
bash tools/clock_pass.sh || exit 1
cp gpurun_out/clock_pass.json gpurun_out/prof_r05/keep/r05_clock_pass.json
timeout -k 10 200 python -u tools/step_parts.py > gpurun_out/r05_step_parts.json || exit 1
cat gpurun_out/r05_step_parts.json
