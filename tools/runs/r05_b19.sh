# round-5 check 19: table traceback -- its tests, the parity suites that walk R = 1 pairs, then the
# headline / local / dna8k / protein4k bench lines and a kernel trace of the headline
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tb_tables.py > gpurun_out/b19_tests.log 2>&1 || { tail -30 gpurun_out/b19_tests.log; exit 1; }
tail -2 gpurun_out/b19_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_band_fill.py tests/test_batch_abi.py > gpurun_out/b19_tests2.log 2>&1 || { tail -30 gpurun_out/b19_tests2.log; exit 1; }
tail -2 gpurun_out/b19_tests2.log
bash tools/ab.sh -w "headline local dna8k protein4k" || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b19 -o b19 -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b19_prof.log 2>&1 || { tail gpurun_out/b19_prof.log; exit 1; }
find gpurun_out/prof_b19 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
