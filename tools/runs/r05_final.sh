# round-5 final evidence: full GPU suite, smoke, rocprofv3 trace + WRITE/FETCH PMC of every bench
# workload with the default bench line (tools/profile_all.sh), the batch line, the harness modes
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 1500 bash tools/profile_all.sh r5f || exit 1
for w in batch local dna8k protein4k; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/final_bench_$w.json 2> gpurun_out/final_bench_$w.err || { tail gpurun_out/final_bench_$w.err; exit 1; }
done
timeout -k 10 1500 bash tools/harness.sh r5f > gpurun_out/final_harness.log 2>&1 || { tail -20 gpurun_out/final_harness.log; exit 1; }
echo final done
