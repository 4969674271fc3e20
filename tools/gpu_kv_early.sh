# model / DP / parity tests on the current build, then the interleaved step A/B of MIT_KV_DW_EARLY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_dist_gpu.py tests/test_bf16_parity_gpu.py tests/test_boundary_gpu.py tests/test_plan_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/tkv.log 2>&1; rc=$?; tail -2 gpurun_out/tkv.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh -r 3 "MIT_KV_DW_EARLY=0" "MIT_KV_DW_EARLY=1"
