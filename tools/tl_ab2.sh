#!/bin/bash
# A/B of fill builds: clk/step on a 4-strip chain (m=256) and the headline fill, per library
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = prod ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  SA_HIP_LIB=$L timeout -k 10 60 python tools/timeline.py --n 32768 --m 256 --mode ${TL_MODE:-0} > gpurun_out/tl2_$v.json 2>/dev/null || { echo "timeline $v failed"; exit 1; }
  SA_HIP_LIB=$L timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode ${TL_MODE:-0} > gpurun_out/tl3_$v.json 2>/dev/null || { echo "timeline $v failed"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/tl2_$v.json')); e=json.load(open('gpurun_out/tl3_$v.json'))
print('$v', 'm256', d['ns_per_step_by_strip'], d['clk_per_step_mean'], '| 32k', {k: e[k] for k in ('total_us','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean')})"
done
