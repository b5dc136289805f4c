set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 1 > gpurun_out/tl_local_new.json 2>/dev/null &&
timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 0 > gpurun_out/tl_global_new.json 2>/dev/null
