# round-4 check 22 (final build): GPU suite, smoke, bench lines of every workload (v5), rocprofv3 trace +
# PMC of every workload and the default bench line with its CPU baseline
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b22_tests.log 2>&1 || { tail -n 40 gpurun_out/b22_tests.log; exit 1; }
tail -n 2 gpurun_out/b22_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for w in headline local dna8k protein4k batch; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${w}_v5.json 2> gpurun_out/b22_$w.err || { tail -n 20 gpurun_out/b22_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/bench_${w}_v5.json | cut -c1-150
done
bash tools/profile_all.sh b22 | cut -c1-400
