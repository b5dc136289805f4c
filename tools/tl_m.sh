for m in 64 128 256 1024; do
  timeout -k 10 60 python tools/timeline.py --n 32768 --m $m > gpurun_out/tlm_$m.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/tlm_$m.json'))
print($m, {k: d[k] for k in ('total_us','clk_per_step_mean','ns_per_step_by_strip','lag_ns_in_group_mean')})"
done
