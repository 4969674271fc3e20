#!/bin/bash
# Build libmit_hip.so from the kernel sources of a git revision into lib/ab/libmit_hip_NAME.so, for a same-box
# A/B against the working tree (MIT_LIB=..., tools/gpu_ab.sh / tools/gpu_ab_lib.sh). The C ABI must match the
# binding's ABI_VERSION. Usage: tools/build_rev_lib.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TMP=$(mktemp -d /tmp/revlib.XXXXXX)
git -C "$ROOT" archive "$REV" multimodal-image-transformer_amd/csrc include | tar -x -C "$TMP"
make -C "$TMP/multimodal-image-transformer_amd/csrc" -j8 ../lib/libmit_hip.so > /dev/null
mkdir -p "$ROOT/multimodal-image-transformer_amd/lib/ab"
cp "$TMP/multimodal-image-transformer_amd/lib/libmit_hip.so" "$ROOT/multimodal-image-transformer_amd/lib/ab/libmit_hip_$NAME.so"
rm -rf "$TMP"
echo "built lib/ab/libmit_hip_$NAME.so from $REV"
