cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/tln.log 2>&1; rc=$?; tail -2 gpurun_out/tln.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh -r 3 "MIT_LN_RW=2" "MIT_LN_RW=1"
