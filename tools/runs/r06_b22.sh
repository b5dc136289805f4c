# round 6: the batch step with its fill stream (encode + fill) at high priority (SA_BENCH_FILL_PRIO):
# the next step's encode no longer queues behind the traceback's workgroups
mkdir -p gpurun_out
: > gpurun_out/ab.log
for rep in 1 2 3; do
  for pr in 0 1; do
    SA_BENCH_FILL_PRIO=$pr LABEL=prio$pr timeout -k 10 600 bash tools/ab.sh -w "batch" -s 20 > /dev/null || exit 1
  done
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b22_ab.log
