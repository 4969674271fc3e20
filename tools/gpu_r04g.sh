# r04g: split-K epilogue A/B + step parts, then the round's evidence (full -m gpu suite, bench line,
# rocprofv3 passes of tools/profile_round.sh, decode / CLIP-L workload lines)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04g
V=multimodal-image-transformer_amd/lib/ab/libmit_hip_nosplitepi.so
B="--no-cpu-baseline --no-also --no-roofline --steps 30 --warmup 5"
for r in 1 2; do
  echo "## split $(timeout -k 10 200 python -u bench.py $B | cut -c90-150)"
  echo "## nosplit $(MIT_LIB=$V timeout -k 10 200 python -u bench.py $B | cut -c90-150)"
done
timeout -k 10 200 python -u tools/step_parts.py || exit 1
MIT_LIB=$V timeout -k 10 200 python -u tools/step_parts.py || exit 1
timeout -k 10 200 python -u bench.py --workload decode --no-cpu-baseline > gpurun_out/r04g/decode.json 2>&1 || exit 1
tail -1 gpurun_out/r04g/decode.json | cut -c1-220
bash tools/gpu_round.sh r04
