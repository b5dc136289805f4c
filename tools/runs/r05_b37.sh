# round-5 check 37: table kernel chains in lockstep per thread, all staging loads in flight: table
# tests, phase times, bench lines
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tb_tables.py tests/test_band_fill.py tests/test_edge_cases.py > gpurun_out/b37_tests.log 2>&1 || { tail -30 gpurun_out/b37_tests.log; exit 1; }
tail -1 gpurun_out/b37_tests.log
bash tools/runs/r05_b25.sh | cut -c1-330 || exit 1
bash tools/ab.sh -w "headline local dna8k protein4k" || exit 1
