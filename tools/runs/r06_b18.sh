# round 6: strip tables of 1024 threads when every strip has a CU (SA_TB_WIDE): the table traceback
# tests, then same-box A/Bs of the traceback of the small single pairs
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_tb_tables.py tests/test_edge_cases.py > gpurun_out/r6b18_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b18_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b18_tests.log
: > gpurun_out/ab.log
for rep in 1 2 3; do
  for wd in 1 0; do
    SA_TB_WIDE=$wd LABEL=wide$wd timeout -k 10 600 bash tools/ab.sh -w "dna8k protein4k" -s 20 > /dev/null || exit 1
  done
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b18_ab.log
