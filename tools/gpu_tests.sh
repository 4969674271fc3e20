# GPU check: the -m gpu suite, then the bf16 parity table (tools/bf16_parity_report.py).
# A test failure (rc 1) still runs the report; any other status (fault, abort, timeout) stops.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${MIT_PYTEST_ARGS} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ -n "${MIT_SKIP_REPORT}" ]; then exit $rc; fi
timeout -k 10 600 python -u tools/bf16_parity_report.py > gpurun_out/parity.log 2>&1
rc2=$?
tail -5 gpurun_out/parity.log
exit $(( rc > rc2 ? rc : rc2 ))
