#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY. Compiles the reference's OWN test driver, tests/tests.cu (Catch2), as
# C++14 against THIS repository's include/SequenceAlignment.hpp and links it with our
# libsequence_alignment.so / libsa_hip.so: the reference's callers, unchanged, on our API.
#
# tests.cu includes "../SequenceAlignment.hpp" (tests/tests.cu:10), so the scratch directory (in
# /tmp, outside the repository) holds our header at its root and the reference's tests.cu and
# catch.hpp under tests/. -DCATCH_CONFIG_NO_POSIX_SIGNALS: Catch 2.13's sigaltstack size is not a
# constant on glibc 2.35. Output: oracle/_ref/ref_tests_api (git-ignored; it travels to the GPU
# box). tests/benchmarks.cu is NOT built: it #includes tests/old_alignSequenceGPU.cu (CUDA kernels)
# and calls cudaGetDeviceProperties, so it needs nvcc; the -DBENCHMARK macro contract it relies on
# is checked by bin/sa_benchmark_contract instead (csrc/host/benchmark_contract.cpp).
set -euo pipefail
REF=${SA_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/.." && pwd)
OUT="$HERE/_ref"
if [ ! -f "$REF/tests/tests.cu" ]; then
    echo "build_ref_callers.sh: reference not present at $REF; skipping (prebuilt $OUT is used if present)" >&2
    exit 0
fi
SCRATCH=$(mktemp -d /tmp/sa_ref_callers.XXXXXX)
trap 'rm -rf "$SCRATCH"' EXIT
mkdir -p "$SCRATCH/tests" "$OUT"
cp "$REF/tests/tests.cu" "$REF/tests/catch.hpp" "$SCRATCH/tests/"
cp "$ROOT/include/SequenceAlignment.hpp" "$SCRATCH/"
LIB="$ROOT/sequence-alignment-gpu_amd/lib"
g++ -std=c++14 -O1 -DCATCH_CONFIG_NO_POSIX_SIGNALS -I"$ROOT/include" -x c++ "$SCRATCH/tests/tests.cu" \
    -L"$LIB" -lsequence_alignment -lsa_hip -Wl,-rpath,'$ORIGIN/../../sequence-alignment-gpu_amd/lib' \
    -o "$OUT/ref_tests_api"
echo "built $OUT/ref_tests_api"
