#!/bin/bash
# batch workload: plans per rank (traceback of chunk k overlapping the fill of chunk k+1)
mkdir -p gpurun_out; : > gpurun_out/swc.log
for c in ${CHUNKS:-1 2 4 8}; do
  echo "== chunks=$c" >> gpurun_out/swc.log
  timeout -k 10 120 python bench.py --workload batch --batch-chunks $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/swc_tmp.log 2>&1 || { cat gpurun_out/swc_tmp.log; exit 1; }
  python tools/show_bench.py gpurun_out/swc_tmp.log >> gpurun_out/swc.log
  python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/swc_tmp.log') if l.startswith('{')][0]; print('  pair0', d['sample_result'], 'fill span', d['fill_ms_per_launch'])" >> gpurun_out/swc.log
done
cat gpurun_out/swc.log
