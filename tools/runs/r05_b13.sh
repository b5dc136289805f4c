# round-5 check 13: local walk with the pending check before the record store: parity subset, then
# local / headline bench lines against base0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_edge_cases.py tests/test_batch_golden.py -m gpu -x -q --timeout 60 --timeout-method thread > gpurun_out/r5b13_tests.log 2>&1 || { tail -n 40 gpurun_out/r5b13_tests.log; exit 1; }
tail -n 1 gpurun_out/r5b13_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 600 bash tools/ab.sh -l "base0 base" -w "local headline" -s 20 > /dev/null || exit 1
done
cut -c1-150 gpurun_out/ab.log
