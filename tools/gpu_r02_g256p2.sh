# Persistent 256 GEMM round 2: tests on the default build, isolated A/B on it and on the no-swap
# timing variant (operand order as the one-tile kernel)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/g256p2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm256p_ab.py > $OUT/ab.txt 2>&1 && cat $OUT/ab.txt &&
MIT_LIB=multimodal-image-transformer_amd/lib/variants/libmit_hip_noswap.so timeout -k 10 300 python -u tools/gemm256p_ab.py > $OUT/ab_noswap.txt 2>&1 && cat $OUT/ab_noswap.txt
