# gemm256 epilogue check: the GEMM tests, store-pattern microbenchmark, per-phase stamps and the
# encoder-shape timings of the current build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t256.log 2>&1; rc=$?; tail -3 gpurun_out/t256.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/store_bench > gpurun_out/store_bench.txt 2>&1 || { tail -3 gpurun_out/store_bench.txt; exit 1; }
MIT_LIB=multimodal-image-transformer_amd/lib/variants/libmit_hip_stamp.so timeout -k 10 100 python -u tools/g256_stamps.py iso8 iso64 enc_qkv+bias enc_o+res enc_fc1+gelu > gpurun_out/st_dpp.txt 2>&1 || { tail -5 gpurun_out/st_dpp.txt; exit 1; }
grep -E "==|epilogue  " gpurun_out/st_dpp.txt
GEMM_SHAPES="enc_qkv+bias,enc_o+res,enc_fc1+gelu,enc_fc2+res,dec_kv_all,dec_fc_out,clip_qkv,clip_o+res,clip_fc1+gelu,clip_fc2+res" timeout -k 10 200 python -u tools/gemm_bench.py 2
