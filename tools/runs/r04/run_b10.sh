# round-4 check 10: band start-up stamps; wait-loop sleep A/B (sleep 1 = bst, none = bs0, 8 = bs8) and
# feed prefetch step (10 = bst, 13 = bp13, 15 = bp15)
mkdir -p gpurun_out
: > gpurun_out/b10.log
for rep in 1 2; do
  for lib in bst bx bs0 bs8 bp13 bp15; do
    for mode in 0 1; do
      echo "$lib mode=$mode " >> gpurun_out/b10.log
      SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 120 python tools/band_stamps.py 32768 $mode 2>/dev/null | grep "^{" >> gpurun_out/b10.log || { echo failed $lib; exit 1; }
    done
  done
done
cat gpurun_out/b10.log
