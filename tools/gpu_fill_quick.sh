#!/bin/bash
# quick fill check: parity tests of the chained R = 1 fill + timelines (global / local 32k)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_quick.log 2>&1 &&
timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 0 > gpurun_out/tl_g.json 2>/dev/null &&
timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 1 > gpurun_out/tl_l.json 2>/dev/null &&
timeout -k 10 60 python tools/timeline.py --n 32768 --m 64 --mode 0 > gpurun_out/tl_g64.json 2>/dev/null
