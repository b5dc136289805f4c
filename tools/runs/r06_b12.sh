# round 6: the pipelined batch with the column walk capped at SA_TB_CAP waves (each walking pairs in
# turn) beside the next fill: parity with the cap, then a same-box A/B of the batch step
mkdir -p gpurun_out
SA_TB_CAP=256 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_batch_golden.py -k "config5_every or local_batch" > gpurun_out/r6b12_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b12_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b12_tests.log
: > gpurun_out/ab.log
for rep in 1 2 3; do
  for cap in 0 256 512 1024; do
    SA_TB_CAP=$cap LABEL=cap$cap timeout -k 10 600 bash tools/ab.sh -w "batch" -s 20 > /dev/null || exit 1
  done
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b12_ab.log
