# round-4 check 25: the touch as its own kernel for DNA-sized alphabets (tk) vs touch for every
# alphabet (cur): band / parity GPU tests on tk, then headline, 8192², protein 4096² bench lines
mkdir -p gpurun_out
SA_HIP_LIB=$PWD/build_exp/libsa_tk.so timeout -k 10 600 python -u -m pytest tests/test_band_fill.py tests/test_gpu_parity.py tests/test_edge_cases.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b25_tests.log 2>&1 || { tail -n 40 gpurun_out/b25_tests.log; exit 1; }
tail -n 2 gpurun_out/b25_tests.log
: > gpurun_out/b25_ab.log
for rep in 1 2; do
  for lib in cur tk; do
    for w in headline dna8k protein4k; do
      SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b25_x.json 2> gpurun_out/b25_x.err || { tail -n 20 gpurun_out/b25_x.err; exit 1; }
      echo "$rep $lib $w $(python tools/show_bench.py gpurun_out/b25_x.json)" >> gpurun_out/b25_ab.log
    done
  done
done
cut -c1-130 gpurun_out/b25_ab.log
