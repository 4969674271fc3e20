# Persistent vs one-tile 256 GEMM with the epilogue compiled out (timing variant): main loops alone
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/g256p3
mkdir -p $OUT
MIT_LIB=multimodal-image-transformer_amd/lib/variants/libmit_hip_noepi.so timeout -k 10 300 python -u tools/gemm256p_ab.py > $OUT/ab_noepi.txt 2>&1 ; cat $OUT/ab_noepi.txt
