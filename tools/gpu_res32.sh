# f32 encoder residual stream: parity of the deep fixtures with and without it, the model tests, then
# the LDS-staged epilogue's step stamps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/res32
for mode in on off; do
  MIT_ENCODER_F32_RESIDUAL=$mode timeout -k 10 300 python -u tools/bf16_parity_report.py cfg1_b2_patches cfg2_b2_patches cfg3_b2_patches tiny_clip336_patches \
    > gpurun_out/res32/parity_$mode.log 2>&1 || { tail -20 gpurun_out/res32/parity_$mode.log; exit 1; }
  cp gpurun_out/bf16_parity.json gpurun_out/res32/parity_$mode.json
  python3 -c "
import json; d=json.load(open('gpurun_out/res32/parity_$mode.json'))
for k,v in d.items():
    b=v['bf16']; print('$mode', k, 'logits_rel %.3e enc %.3e gmed %.3f gmax %.3f' % (b['logits_rel_l2'], b['enc_rel_l2'], b['grad_rms_median'], b['grad_rms_max']))"
done
MIT_ENCODER_F32_RESIDUAL=on timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_bf16_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/res32/tests_on.log 2>&1; tail -3 gpurun_out/res32/tests_on.log
