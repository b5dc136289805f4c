#!/bin/bash
# Per-strip step time along short chains (m = 128 .. 2048), global and local: does a strip run
# slower than the strip above it?
set -e
mkdir -p gpurun_out
for mode in 0 1; do for m in 128 256 512 2048; do
  timeout -k 10 60 python tools/timeline.py --n 32768 --m $m --mode $mode > gpurun_out/tlc_${mode}_$m.json 2>/dev/null
  python -c "
import json; d=json.load(open('gpurun_out/tlc_${mode}_$m.json'))
print($mode, $m, d['total_us'], d['clk_per_step_mean'], d['ns_per_step_by_strip'][:16], d['lag_ns_by_strip'][:16])"
done; done
