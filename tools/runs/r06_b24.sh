# round 6: why the control-word reset slowed the pipelined batch: the product build, the reset with
# the memset launch removed (ctl, as tried), and the reset with the memset kept (both)
mkdir -p gpurun_out
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 900 bash tools/ab.sh -l "base ctl both" -w "batch" -s 20 > /dev/null || exit 1
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b24_ab.log
