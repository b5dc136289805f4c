# round-6 final evidence (2/2): bench lines of every workload, the config-5 shard lines, the
# reference harness modes
set -o pipefail
mkdir -p gpurun_out
for w in batch local dna8k protein4k; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/r6f_bench_$w.json 2> gpurun_out/r6f_bench_$w.err || { tail gpurun_out/r6f_bench_$w.err; exit 1; }
  tail -c 400 gpurun_out/r6f_bench_$w.json
done
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --workload batch --shard-of $n --steps 20 --no-cpu-baseline > gpurun_out/r6f_shard_of_$n.json 2> gpurun_out/r6f_shard_of_$n.err || { tail gpurun_out/r6f_shard_of_$n.err; exit 1; }
done
timeout -k 10 900 bash tools/harness.sh r6f > gpurun_out/r6f_harness_run.log 2>&1 || { tail -20 gpurun_out/r6f_harness_run.log; exit 1; }
echo final_b done
