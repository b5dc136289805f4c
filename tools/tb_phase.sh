#!/bin/bash
# walk phase split (experiment build build_exp/libsa_wt.so): staging vs row walk, global / local 32k
mkdir -p gpurun_out
for mode in 0 1; do
  SA_HIP_LIB=$PWD/build_exp/libsa_wt.so timeout -k 10 120 python tools/tb_timing.py --mode $mode || exit 1
done
