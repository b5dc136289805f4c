#!/bin/bash
# Contention test: short chains (m = 2048, 32 strips) alone and as 4 / 16 concurrent copies
set -e
mkdir -p gpurun_out
for mode in 0 1; do for p in 1 4 16; do
  timeout -k 10 60 python tools/timeline.py --n 32768 --m 2048 --mode $mode --pairs $p > gpurun_out/tlp_${mode}_$p.json 2>/dev/null
  python -c "
import json; d=json.load(open('gpurun_out/tlp_${mode}_$p.json'))
print($mode, $p, d['total_us'], d['clk_per_step_mean'], d['ns_per_step_mean'], d['ns_per_step_max'], d['cus_used'], d['max_strips_on_one_simd_concurrently'])"
done; done
