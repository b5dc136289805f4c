# round-5 check 30: eight rounds past 131072 rows: 250000^2 local, then the full GPU suite
set -o pipefail
LABEL=tb-250000 bash tools/ab.sh -w "headline local" -s 3 -- --size 250000 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/b30_tests.log 2>&1 || { tail -30 gpurun_out/b30_tests.log; exit 1; }
tail -1 gpurun_out/b30_tests.log
