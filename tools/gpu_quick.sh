#!/bin/bash
# GPU box: parity tests, then the latency harness (alignSequenceGPU end to end) at small and large sizes.
tag=${1:-q}
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/gpurun_out"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 40 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 3 gpurun_out/${tag}_tests.log
out=$root/gpurun_out
mkdir -p "$out/${tag}_cwd"
python "$root/tools/score_matrices.py" "$out/${tag}_cwd" || exit 1
cd "$out/${tag}_cwd" || exit 1
for m in global local; do
  timeout -k 10 200 "$root/sequence-alignment-gpu_amd/bin/sa_benchmarks" latency $m --repeats 3 --json > "$out/${tag}_lat_$m.log" 2>&1 || { tail -n 20 "$out/${tag}_lat_$m.log"; exit 1; }
  grep '^{' "$out/${tag}_lat_$m.log"
done
