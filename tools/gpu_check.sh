#!/bin/bash
# GPU box check used during development: parity tests, then the three bench workloads (no CPU
# baseline) -> gpurun_out/<tag>_*.log. Every GPU step has its own time limit; stops at the first failure.
tag=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 40 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 3 gpurun_out/${tag}_tests.log
for w in ${WORKLOADS:-headline local batch dna8k protein4k}; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_$w.log 2>&1 || { tail -n 20 gpurun_out/${tag}_$w.log; exit 1; }
  python tools/show_bench.py gpurun_out/${tag}_$w.log
done
