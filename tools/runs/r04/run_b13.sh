# round-4 check 13: traceback tests on the speculative stager read, then a same-box A/B of the
# traceback against the previous walk (build_exp/libsa_wold.so)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b13_tests.log 2>&1 || { tail -n 40 gpurun_out/b13_tests.log; exit 1; }
tail -n 2 gpurun_out/b13_tests.log
: > gpurun_out/b13_ab.log
for rep in 1 2 3; do
  for lib in new wold; do
    for w in headline local; do
      if [ $lib = wold ]; then export SA_HIP_LIB=$PWD/build_exp/libsa_wold.so; else unset SA_HIP_LIB; fi
      timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b13_x.json 2> gpurun_out/b13_x.err || { tail -n 20 gpurun_out/b13_x.err; exit 1; }
      echo "$rep $lib $w $(python tools/show_bench.py gpurun_out/b13_x.json)" >> gpurun_out/b13_ab.log
    done
  done
done
unset SA_HIP_LIB
cat gpurun_out/b13_ab.log
