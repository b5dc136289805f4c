# round-5 check 2: band second feed read (pf2) and per-quad band LDS addresses (pq = both, pqn = per-quad
# only): band/parity GPU tests on pq, then same-box A/B against the round-start build (base0)
mkdir -p gpurun_out
timeout -k 10 60 tools/microbench/bandbench > gpurun_out/bandbench_2w.log 2>&1 && cat gpurun_out/bandbench_2w.log
SA_HIP_LIB=$PWD/build_exp/libsa_pq.so timeout -k 10 400 python -u -m pytest tests/test_band_fill.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b2_tests.log 2>&1 || { tail -n 30 gpurun_out/r5b2_tests.log; exit 1; }
tail -n 1 gpurun_out/r5b2_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 600 bash tools/ab.sh -l "base0 pf2 pqn pq" -w "headline local dna8k" -s 20 > /dev/null || exit 1
done
cut -c1-150 gpurun_out/ab.log
