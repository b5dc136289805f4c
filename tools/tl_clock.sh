#!/bin/bash
# Timeline with shader-clock stamps: effective clock, clocks per step and SIMD sharing, lone strip
# vs full chain, with and without one chain workgroup per CU (SA_CHAIN_LDS_KB).
mkdir -p gpurun_out
: > gpurun_out/tlc.log
for c in "64 4 0" "256 4 0" "32768 4 0" "32768 4 96"; do set -- $c
  echo "== m=$1 waves=$2 lds_kb=$3" >> gpurun_out/tlc.log
  SA_CHAIN_LDS_KB=$3 timeout -k 10 60 python tools/timeline.py --n 32768 --m $1 --waves $2 >> gpurun_out/tlc.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/tlc.log
