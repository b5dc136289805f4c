#!/bin/bash
# One GPU call: rocprofv3 trace + PMC passes for the three bench workloads, then the default bench
# line with its CPU baseline. Usage: tools/profile_all.sh <tag>
tag=${1:-run}
set -o pipefail
mkdir -p gpurun_out
bash tools/profile.sh ${tag}_headline --workload headline --no-cpu-baseline --steps 5 --warmup 1 || exit 1
bash tools/profile.sh ${tag}_batch --workload batch --no-cpu-baseline --steps 5 --warmup 1 || exit 1
bash tools/profile.sh ${tag}_local --workload local --no-cpu-baseline --steps 5 --warmup 1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench_default.json 2> gpurun_out/${tag}_bench_default.err || exit 1
cat gpurun_out/${tag}_bench_default.json
