#!/bin/bash
# timeline of experiment builds (build_exp/libsa_<tag>.so; "base" = the product library)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  for c in "256 4" "128 1" "32768 4"; do set -- $c
    echo "== $v m=$1 waves=$2" >> gpurun_out/tlx.log
    SA_HIP_LIB=$L timeout -k 10 60 python tools/timeline.py --n 32768 --m $1 --waves $2 >> gpurun_out/tlx.log 2>&1 || exit 1
  done
done
