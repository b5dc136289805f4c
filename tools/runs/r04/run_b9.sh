# round-4 check 9: GPU suite, band start-up stamps (experiment build), bench lines of all workloads
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b9_tests.log 2>&1 || { tail -n 40 gpurun_out/b9_tests.log; exit 1; }
tail -n 2 gpurun_out/b9_tests.log
for mode in 0 1; do
  SA_HIP_LIB=$PWD/build_exp/libsa_bst.so timeout -k 10 120 python tools/band_stamps.py 32768 $mode > gpurun_out/b9_stamps_$mode.log 2>&1 || { tail -20 gpurun_out/b9_stamps_$mode.log; exit 1; }
  cat gpurun_out/b9_stamps_$mode.log
done
for w in headline local dna8k protein4k batch; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b9_$w.json 2> gpurun_out/b9_$w.err || { tail -n 20 gpurun_out/b9_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/b9_$w.json
done
