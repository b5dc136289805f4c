# round 6: the batch step with the traceback on CUs of its own (stream CU masks, SA_BENCH_TB_CUS) and
# the new copy-0 profile test
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_band_fill.py -k copy0 > gpurun_out/r6b15_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b15_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b15_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  for c in 0 8 16 32; do
    SA_BENCH_TB_CUS=$c LABEL=tbcus$c timeout -k 10 600 bash tools/ab.sh -w "batch" -s 20 > /dev/null || exit 1
  done
  SA_BENCH_TB_CUS=16 SA_TB_CAP=256 LABEL=tbcus16cap256 timeout -k 10 600 bash tools/ab.sh -w "batch" -s 20 > /dev/null || exit 1
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b15_ab.log
