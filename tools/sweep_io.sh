#!/bin/bash
# headline fill vs the I/O wave's idle poll period (SA_IO_SLEEP, units of s_sleep 1 = 64 clocks)
mkdir -p gpurun_out; : > gpurun_out/swio.log
for v in ${IOS:-0 1 2 4 8}; do
  echo "== io_sleep=$v" >> gpurun_out/swio.log
  SA_IO_SLEEP=$v timeout -k 10 120 python bench.py --workload headline --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/swio_tmp.log 2>&1 || { cat gpurun_out/swio_tmp.log; exit 1; }
  python tools/show_bench.py gpurun_out/swio_tmp.log >> gpurun_out/swio.log
done
cat gpurun_out/swio.log
