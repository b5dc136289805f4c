# round-5 check 40: random sweep of the table traceback against the oracle (one and four rounds)
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tb_tables.py > gpurun_out/b40_tests.log 2>&1 || { tail -30 gpurun_out/b40_tests.log; exit 1; }
grep -c PASSED gpurun_out/b40_tests.log; tail -1 gpurun_out/b40_tests.log
