# round-4 check 24: band code touch 6 bodies ahead for every alphabet (cur) vs DNA only, protein
# touching its own columns (ng): headline, 8192², protein 4096² bench lines, two repetitions
mkdir -p gpurun_out
: > gpurun_out/b24_ab.log
for rep in 1 2; do
  for lib in cur ng; do
    for w in headline dna8k protein4k; do
      SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b24_x.json 2> gpurun_out/b24_x.err || { tail -n 20 gpurun_out/b24_x.err; exit 1; }
      echo "$rep $lib $w $(python tools/show_bench.py gpurun_out/b24_x.json)" >> gpurun_out/b24_ab.log
    done
  done
done
cut -c1-150 gpurun_out/b24_ab.log
