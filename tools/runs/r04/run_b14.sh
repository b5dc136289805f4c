# round-4 check 14: GPU suite, walk A/B (local-only speculative stager read vs previous walk), bench
# lines of every workload (v4)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b14_tests.log 2>&1 || { tail -n 40 gpurun_out/b14_tests.log; exit 1; }
tail -n 2 gpurun_out/b14_tests.log
: > gpurun_out/b14_ab.log
for rep in 1 2; do
  for lib in new wold; do
    for w in headline local; do
      if [ $lib = wold ]; then export SA_HIP_LIB=$PWD/build_exp/libsa_wold.so; else unset SA_HIP_LIB; fi
      timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b14_x.json 2> gpurun_out/b14_x.err || { tail -n 20 gpurun_out/b14_x.err; exit 1; }
      echo "$rep $lib $w $(python tools/show_bench.py gpurun_out/b14_x.json)" >> gpurun_out/b14_ab.log
    done
  done
done
unset SA_HIP_LIB
cat gpurun_out/b14_ab.log
for w in headline local dna8k protein4k batch; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${w}_v4.json 2> gpurun_out/b14_$w.err || { tail -n 20 gpurun_out/b14_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/bench_${w}_v4.json
done
