# round-4 check 11: band feed misses (counters only) with the feed read at step 10 / 13 / 15
mkdir -p gpurun_out
: > gpurun_out/b11.log
for rep in 1 2; do
  for lib in bm bxm bm13 bm15; do
    for mode in 0 1; do
      echo "$lib mode=$mode " >> gpurun_out/b11.log
      SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 120 python tools/band_miss.py 32768 $mode 2>/dev/null | grep "^{" >> gpurun_out/b11.log || { echo failed $lib; exit 1; }
    done
  done
done
cat gpurun_out/b11.log
