# round-5 check 26: table kernel slow path on the staged masks (unknown past them), 512-thread blocks:
# table tests, phase times, bench lines
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tb_tables.py tests/test_band_fill.py > gpurun_out/b26_tests.log 2>&1 || { tail -30 gpurun_out/b26_tests.log; exit 1; }
tail -1 gpurun_out/b26_tests.log
bash tools/runs/r05_b25.sh | cut -c1-400 || exit 1
bash tools/ab.sh -w "headline local dna8k protein4k" || exit 1
