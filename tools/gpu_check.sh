#!/bin/bash
# GPU box development check: the -m gpu suite (parity + edge cases), the bench workloads without
# the CPU baseline, then the chained-fill timeline. Every GPU step has its own time limit and the
# script stops at the first failure. Output: gpurun_out/<tag>_*.
#   tools/gpu_check.sh [tag]      WORKLOADS="headline local" to change the bench list;
#                                 GENERIC=1 also runs the traceback parity subset with the C++ line loop
tag=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 ||
  { tail -n 40 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 2 gpurun_out/${tag}_tests.log
if [ -n "$GENERIC" ]; then
  sel="test_known_answers or test_data_pairs or test_random_pairs or test_seeded_vs_oracle or test_batch_plan_config5 or test_gap_pairs"
  SA_TB_GENERIC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$sel" \
    > gpurun_out/${tag}_generic.log 2>&1 || { tail -n 40 gpurun_out/${tag}_generic.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_generic.log
fi
for w in ${WORKLOADS:-headline local dna8k protein4k batch}; do
  timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${tag}_$w.json 2> gpurun_out/${tag}_$w.err ||
    { tail -n 20 gpurun_out/${tag}_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/${tag}_$w.json
done
[ -n "$NO_TIMELINE" ] || bash tools/timeline.sh -m "32768 64 256"
