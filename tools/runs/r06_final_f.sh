# round-6 final build (staging kernel, wide strip tables; the control-word reset reverted): the full
# GPU suite, smoke, the default bench line, the other workloads' bench lines, the harness modes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6j_tests.log 2>&1 || { tail -30 gpurun_out/r6j_tests.log; exit 1; }
tail -1 gpurun_out/r6j_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6j_smoke.log 2>&1 || { tail gpurun_out/r6j_smoke.log; exit 1; }
tail -1 gpurun_out/r6j_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r6j_bench_default.json 2> gpurun_out/r6j_bench_default.err || exit 1
for w in batch local dna8k protein4k; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/r6j_bench_$w.json 2> gpurun_out/r6j_bench_$w.err || { tail gpurun_out/r6j_bench_$w.err; exit 1; }
done
timeout -k 10 900 bash tools/harness.sh r6j > gpurun_out/r6j_harness_run.log 2>&1 || { tail -20 gpurun_out/r6j_harness_run.log; exit 1; }
echo final_f done
