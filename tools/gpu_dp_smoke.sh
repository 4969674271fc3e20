# The bench's N>1 code path exactly as the driver runs it (torchrun, default flags: native replay,
# DataParallel buckets on the side stream, encoder prefetch, loss all-reduce, roofline probe) on ONE
# GPU: 2 ranks over gloo sharing cuda:0 (RCCL needs one GPU per rank). Output: gpurun_out/dp2_gloo.*
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MIT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
  > gpurun_out/dp2_gloo.json 2> gpurun_out/dp2_gloo.err
rc=$?; cat gpurun_out/dp2_gloo.json; tail -5 gpurun_out/dp2_gloo.err; exit $rc
