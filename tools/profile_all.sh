#!/bin/bash
# One GPU call: rocprofv3 trace + PMC passes for every bench workload, then the default bench line
# with its CPU baseline. Usage: tools/profile_all.sh <tag> ; WORKLOADS overrides the list.
tag=${1:-run}
set -o pipefail
mkdir -p gpurun_out
for w in ${WORKLOADS:-headline batch local dna8k protein4k}; do
  bash tools/profile.sh ${tag}_$w --workload $w --no-cpu-baseline --steps 5 --warmup 1 || exit 1
done
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench_default.json 2> gpurun_out/${tag}_bench_default.err || exit 1
cat gpurun_out/${tag}_bench_default.json
