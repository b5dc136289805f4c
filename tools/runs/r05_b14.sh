# round-5 check 14 (build c8a00aa + fixes): GPU suite, smoke, bench lines of every workload, the
# reference harness modes, rocprofv3 trace + PMC of every workload and the default bench line
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b14_tests.log 2>&1 || { tail -n 40 gpurun_out/b14_tests.log; exit 1; }
tail -n 1 gpurun_out/b14_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for w in headline local dna8k protein4k batch; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${w}_r5v1.json 2> gpurun_out/b14_$w.err || { tail -n 20 gpurun_out/b14_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/bench_${w}_r5v1.json | cut -c1-150
done
timeout -k 10 1200 bash tools/harness.sh r5v1 > /dev/null || exit 1
tail -n 12 gpurun_out/r5v1_harness.jsonl | cut -c1-200
bash tools/profile_all.sh r5b14 | cut -c1-300
