#!/bin/bash
# GPU box check of the traceback: the whole -m gpu suite (unrolled walk), the per-R parity subset
# with the generic line loop, then bench e2e numbers. Stops at the first failure.
tag=${1:-tb}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_fast.log 2>&1 || { tail -n 40 gpurun_out/${tag}_fast.log; exit 1; }
tail -n 2 gpurun_out/${tag}_fast.log
sel="test_known_answers or test_data_pairs or test_random_pairs or test_seeded_vs_oracle or test_batch_plan_config5 or test_pair_packed"
SA_TB_GENERIC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "$sel" > gpurun_out/${tag}_generic.log 2>&1 || { tail -n 40 gpurun_out/${tag}_generic.log; exit 1; }
tail -n 2 gpurun_out/${tag}_generic.log
for w in ${WORKLOADS:-headline local batch}; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${tag}_$w.log 2>&1 || { tail -n 20 gpurun_out/${tag}_$w.log; exit 1; }
  python tools/show_bench.py gpurun_out/${tag}_$w.log
done
