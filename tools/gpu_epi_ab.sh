cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t256.log 2>&1; rc=$?; tail -3 gpurun_out/t256.log; [ $rc -eq 0 ] || exit $rc
for v in stamp stampl2 stampl4; do echo "#### $v"; MIT_LIB=multimodal-image-transformer_amd/lib/variants/libmit_hip_$v.so timeout -k 10 100 python -u tools/g256_stamps.py iso64 enc_qkv+bias enc_o+res enc_fc1+gelu > gpurun_out/st_$v.txt 2>&1 || { tail -5 gpurun_out/st_$v.txt; exit 1; }; grep -E "==|epilogue  " gpurun_out/st_$v.txt; done
GEMM_SHAPES="enc_qkv+bias,enc_o+res,enc_fc1+gelu,enc_fc2+res,dec_kv_all,dec_fc_out" timeout -k 10 200 python -u tools/gemm_bench.py 2 
