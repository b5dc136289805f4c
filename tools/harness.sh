#!/bin/bash
# Runs sa_benchmarks (the reference's tests/benchmarks.cu modes) on the GPU box from a scratch cwd
# holding scoreMatrices/, one JSON line per size -> gpurun_out/<tag>_harness.jsonl (human-readable
# output in gpurun_out/<tag>_harness.log). Every run has its own time limit; stops at the first failure.
tag=${1:-harness}
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/gpurun_out
bin=$root/sequence-alignment-gpu_amd/bin/sa_benchmarks
mkdir -p "$out" "$out/${tag}_cwd"
python "$root/tools/score_matrices.py" "$out/${tag}_cwd" || exit 1
cd "$out/${tag}_cwd" || exit 1
: > "$out/${tag}_harness.log"
run() {
  local limit=$1; shift
  echo "== $*" | tee -a "$out/${tag}_harness.log"
  timeout -k 10 "$limit" "$bin" "$@" --json >> "$out/${tag}_harness.log" 2>&1 || { echo "FAILED ($?): $*"; tail -n 20 "$out/${tag}_harness.log"; exit 1; }
}
run 240 throughput global --repeats 3
run 240 throughput local --repeats 3
run 240 latency global --repeats 2
run 240 latency local --repeats 2
run 240 batch 8 global
run 240 batch 8 local
run 300 maxlength local
run 300 maxlength global
grep '^{' "$out/${tag}_harness.log" > "$out/${tag}_harness.jsonl"
cat "$out/${tag}_harness.jsonl"
