# round-5 check 24: local table traceback, per-row mask probe: GPU tests, bench
# lines, kernel traces
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tb_tables.py > gpurun_out/b24_tests.log 2>&1 || { tail -30 gpurun_out/b24_tests.log; exit 1; }
tail -1 gpurun_out/b24_tests.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/b24_tests2.log 2>&1 || { tail -30 gpurun_out/b24_tests2.log; exit 1; }
tail -1 gpurun_out/b24_tests2.log
bash tools/ab.sh -w "headline local dna8k protein4k batch" || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in headline dna8k; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b24_$w -o run -- python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b24_$w.log 2>&1 || { tail gpurun_out/b24_$w.log; exit 1; }
f=$(find gpurun_out/prof_b24_$w -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-150
done
