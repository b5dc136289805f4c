# round-5 check 31: the reference's harness modes on the current build
set -o pipefail
timeout -k 10 1500 bash tools/harness.sh r5v2 > gpurun_out/b31.log 2>&1 || { tail -20 gpurun_out/b31.log; exit 1; }
cat gpurun_out/r5v2_harness.jsonl | grep -v '"throughput"'
