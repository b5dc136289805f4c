set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "local_best_cell" --timeout 120 --timeout-method thread > gpurun_out/t_local.log 2>&1 &&
timeout -k 10 300 python bench.py --workload local --steps 10 --warmup 2 > gpurun_out/bench_local.json 2> gpurun_out/bench_local.err
