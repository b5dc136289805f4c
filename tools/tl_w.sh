#!/bin/bash
# timeline + headline fill for W compute waves per chain workgroup
for w in ${WS:-4 8}; do
  SA_WAVES_PER_GROUP=$w timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --waves $w > gpurun_out/tlw_$w.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/tlw_$w.json'))
print('W=$w', {k: d[k] for k in ('total_us','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean','max_strips_on_one_simd_concurrently')})"
  SA_WAVES_PER_GROUP=$w timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bw_$w.json 2>/dev/null || exit 1
  python tools/show_bench.py gpurun_out/bw_$w.json
done
