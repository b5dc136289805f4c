# round-5 check 29: rounds of tables re-centred at the failure point: tests, large-size traceback
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tb_tables.py > gpurun_out/b29_tests.log 2>&1 || { tail -30 gpurun_out/b29_tests.log; exit 1; }
grep -c PASSED gpurun_out/b29_tests.log
for s in 250000 500000; do
  LABEL=tb-$s bash tools/ab.sh -w "headline local" -s 3 -- --size $s || exit 1
done
LABEL=tb-32768 bash tools/ab.sh -w "headline local" || exit 1
