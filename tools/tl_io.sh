for s in 4 1 0; do
  SA_IO_SLEEP=$s timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 > gpurun_out/tlio_$s.json 2>/dev/null || exit 1
  python -c "
import json; e=json.load(open('gpurun_out/tlio_$s.json'))
print('io_sleep=$s', {k: e[k] for k in ('total_us','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean')})"
done
