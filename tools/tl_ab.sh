#!/bin/bash
# A/B of fill builds on the GPU box: per-strip timeline (32768^2, R=1) and the fill time of the
# headline bench for each library. Args: experiment tags (build_exp/libsa_<tag>.so; "prod" = the
# product library). Output: gpurun_out/tlab.log
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = prod ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  echo "== $v" | tee -a gpurun_out/tlab.log
  SA_HIP_LIB=$L timeout -k 10 60 python tools/timeline.py --n 32768 --m ${TL_M:-32768} --mode ${TL_MODE:-0} > gpurun_out/tl_$v.json 2>/dev/null || { echo "timeline $v failed"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/tl_$v.json'))
print({k: d[k] for k in ('total_us','ns_per_step_mean','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean','shader_mhz_mean')})" | tee -a gpurun_out/tlab.log
  SA_HIP_LIB=$L timeout -k 10 120 python bench.py --workload ${BENCH_WL:-headline} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python tools/show_bench.py gpurun_out/b_$v.json | tee -a gpurun_out/tlab.log
done
