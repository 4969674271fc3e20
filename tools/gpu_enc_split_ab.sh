# prefetch-test with the encoder split, then the interleaved A/B of MIT_ENC_SPLIT / MIT_ENC_GATE
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MIT_ENC_SPLIT=6 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k prefetch --timeout 120 --timeout-method thread > gpurun_out/tpf.log 2>&1; rc=$?; tail -3 gpurun_out/tpf.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh -r 2 "MIT_ENC_SPLIT=-1" "MIT_ENC_SPLIT=6" "MIT_ENC_SPLIT=9" "MIT_ENC_SPLIT=11 MIT_ENC_GATE=bwd"
