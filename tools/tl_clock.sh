#!/bin/bash
# Timeline with shader-clock stamps: clocks per step and hand-off lags for growing chains.
mkdir -p gpurun_out
: > gpurun_out/tlc.log
for m in ${MS:-64 256 1024 4096 32768}; do
  echo "== m=$m" >> gpurun_out/tlc.log
  timeout -k 10 60 python tools/timeline.py --n 32768 --m $m --waves 4 2>&1 | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('total_us','ns_per_step_mean','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean','ns_per_step_by_strip')})" >> gpurun_out/tlc.log || exit 1
done
cat gpurun_out/tlc.log
