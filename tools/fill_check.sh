#!/bin/bash
# GPU box, fill development loop: cell-by-cell fill parity (R=1 and multi-strip), then headline /
# local bench fill times and the R=1 chained-strip timeline (lag, clk/step).
tag=${1:-f}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu \
  -k "fill_direction_matrix or seeded_vs_oracle or large_configs or random_pairs" > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests.log
for w in ${WORKLOADS:-headline local}; do
  timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_$w.log 2>&1 || { tail -n 20 gpurun_out/${tag}_$w.log; exit 1; }
  python tools/show_bench.py gpurun_out/${tag}_$w.log
done
timeout -k 10 120 python tools/timeline.py --n 32768 --m 32768 > gpurun_out/${tag}_tl.log 2>&1 || { tail -n 20 gpurun_out/${tag}_tl.log; exit 1; }
tail -n 12 gpurun_out/${tag}_tl.log
