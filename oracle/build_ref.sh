#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY. Builds the reference's OWN CPU path into oracle/_ref/ref_align.
#
# The reference is a single-translation-unit C++14 build (SequenceAlignment.hpp:138-140 #includes
# utilities.cpp, alignSequenceCPU.cpp and alignSequenceGPU.cu). Only the last one needs CUDA
# (<cuda.h>, nvcc), which this image does not have, and it is not on the CPU path. The recipe
# therefore compiles the reference's CPU sources as they are, in a scratch directory OUTSIDE the
# repository (/tmp), with the one GPU #include line deleted from the header, and writes only the
# resulting executable into oracle/_ref/ (git-ignored; it travels to the GPU box as a binary).
# No reference source is copied into the repository and nothing is stubbed.
set -euo pipefail
REF=${SA_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -f "$REF/alignSequenceCPU.cpp" ]; then
    echo "build_ref.sh: reference not present at $REF; skipping (prebuilt $OUT is used if present)" >&2
    exit 0
fi
SCRATCH=$(mktemp -d /tmp/sa_ref_build.XXXXXX)
trap 'rm -rf "$SCRATCH"' EXIT
cp "$REF/utilities.cpp" "$REF/alignSequenceCPU.cpp" "$SCRATCH/"
sed '/alignSequenceGPU.cu/d' "$REF/SequenceAlignment.hpp" > "$SCRATCH/SequenceAlignment.hpp"
mkdir -p "$OUT"
g++ -std=c++14 -O2 -I"$SCRATCH" "$HERE/ref_driver.cpp" -o "$OUT/ref_align"
echo "built $OUT/ref_align"
