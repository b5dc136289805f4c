# round 6: the batch step regression (2.4-2.7 -> 3.3 ms): the three engine changes since it was last
# measured, one library each (engine + walk units of each commit over the same fill units)
mkdir -p gpurun_out
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 900 bash tools/ab.sh -l "base pre wide stage" -w "batch" -s 20 > /dev/null || exit 1
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b23_ab.log
