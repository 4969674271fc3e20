# round-5 evidence on the final tree: the -m gpu suite, the bench line (roofline + cpu_baseline + also),
# the rocprofv3 passes (tools/profile_round.sh r05), the long-dispatch clock pass, smoke(), un-profiled
# step parts
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh r05 || exit 1
bash tools/clock_pass.sh || exit 1
cp gpurun_out/clock_pass.json gpurun_out/prof_r05/keep/r05_clock_pass.json
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/r05_smoke.log
timeout -k 10 200 python -u tools/step_parts.py > gpurun_out/r05_step_parts.json || exit 1
cat gpurun_out/r05_step_parts.json
