#!/bin/bash
# traceback timing (bench e2e) of experiment builds build_exp/libsa_<tag>.so ("base" = product)
mkdir -p gpurun_out
for v in "$@"; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  echo "== $v" >> gpurun_out/tbx.log
  SA_HIP_LIB=$L timeout -k 10 120 python bench.py --workload headline --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/tbx.log 2>&1 || exit 1
done
