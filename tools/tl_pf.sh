#!/bin/bash
# feed-read lead ablation: product (read after step 12) vs experiment builds reading after step 13 / 14
mkdir -p gpurun_out
for v in base pf13 pf14; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  for mode in 0 1; do
    SA_HIP_LIB=$L timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode $mode > gpurun_out/tlpf.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/tlpf.json'))
print('$v', $mode, d['total_us'], d['clk_per_step_mean'], d.get('lag_ns_in_group_mean'), d.get('lag_ns_cross_group_mean'))"
  done
done
