# round-5 check 36: window starts staged in LDS for resolve and walk, direct start group (after check 34:
# the finish kernel): table tests, the full GPU suite, bench lines, kernel trace
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tb_tables.py > gpurun_out/b36_tests.log 2>&1 || { tail -30 gpurun_out/b36_tests.log; exit 1; }
tail -1 gpurun_out/b36_tests.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/b36_tests2.log 2>&1 || { tail -30 gpurun_out/b36_tests2.log; exit 1; }
tail -1 gpurun_out/b36_tests2.log
bash tools/ab.sh -w "headline local dna8k protein4k" || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b36 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b36_prof.log 2>&1 || { tail gpurun_out/b36_prof.log; exit 1; }
f=$(find gpurun_out/prof_b36 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-150
