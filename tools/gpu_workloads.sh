# configs[2] / configs[3] one-GPU train workloads + GPU decoder tests at d768 (gpurun from the repo root)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --workload clip336 --steps 10 --warmup 3 > gpurun_out/b_clip336.json 2> gpurun_out/b_clip336.err &&
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 10 --warmup 3 > gpurun_out/b_cfg3.json 2> gpurun_out/b_cfg3.err
