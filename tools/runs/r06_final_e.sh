# round-6 last build (staging kernel, control-word reset in the encode kernel): smoke, the default
# bench line, the bench lines of the other workloads, the reference harness modes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6i_smoke.log 2>&1 || { tail gpurun_out/r6i_smoke.log; exit 1; }
tail -1 gpurun_out/r6i_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r6i_bench_default.json 2> gpurun_out/r6i_bench_default.err || exit 1
for w in batch local dna8k protein4k; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/r6i_bench_$w.json 2> gpurun_out/r6i_bench_$w.err || { tail gpurun_out/r6i_bench_$w.err; exit 1; }
done
timeout -k 10 900 bash tools/harness.sh r6i > gpurun_out/r6i_harness_run.log 2>&1 || { tail -20 gpurun_out/r6i_harness_run.log; exit 1; }
echo final_e done
