# round-4 check 12: GPU suite on the wait-order fix, then a same-box A/B against the previous fill
# (build_exp/libsa_old.so, built from the prior commit's sources)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b12_tests.log 2>&1 || { tail -n 40 gpurun_out/b12_tests.log; exit 1; }
tail -n 2 gpurun_out/b12_tests.log
: > gpurun_out/b12_ab.log
for rep in 1 2 3; do
  for lib in new old; do
    for w in headline local dna8k; do
      if [ $lib = old ]; then export SA_HIP_LIB=$PWD/build_exp/libsa_old.so; else unset SA_HIP_LIB; fi
      timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b12_x.json 2> gpurun_out/b12_x.err || { tail -n 20 gpurun_out/b12_x.err; exit 1; }
      echo "$rep $lib $w $(python tools/show_bench.py gpurun_out/b12_x.json)" >> gpurun_out/b12_ab.log
    done
  done
done
unset SA_HIP_LIB
cat gpurun_out/b12_ab.log
