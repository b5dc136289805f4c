mkdir -p gpurun_out
for M in 32768 64 256; do
timeout -k 10 60 python tools/timeline.py --n 32768 --m $M --mode ${TL_MODE:-0} > gpurun_out/tl_$M.json 2>gpurun_out/tl_err.log || { cat gpurun_out/tl_err.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/tl_$M.json'))
print($M, {k: d.get(k) for k in ('total_us','ns_per_step_mean','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean','shader_mhz_mean')})"
done
