#!/bin/bash
# Fill timelines, global vs local, lone strip (m = 64) and chained (m = 32768): clk/step and lag
set -e
mkdir -p gpurun_out
for mode in 0 1; do for m in 64 32768; do
  timeout -k 10 60 python tools/timeline.py --n 32768 --m $m --mode $mode > gpurun_out/tll_${mode}_$m.json 2>/dev/null
  python -c "
import json; d=json.load(open('gpurun_out/tll_${mode}_$m.json'))
print($mode, $m, {k: d.get(k) for k in ('total_us','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean')})"
done; done
