mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_band_fill.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/b1_band.log 2>&1 || { tail -n 40 gpurun_out/b1_band.log; exit 1; }
tail -n 8 gpurun_out/b1_band.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b1_tests.log 2>&1 || { tail -n 40 gpurun_out/b1_tests.log; exit 1; }
tail -n 3 gpurun_out/b1_tests.log
for w in headline local dna8k protein4k; do
  timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b1_$w.json 2> gpurun_out/b1_$w.err || { tail -n 20 gpurun_out/b1_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/b1_$w.json
done
bash tools/timeline.sh -m "32768" -o "0 1" -f "total_us ns_per_step_mean lag_ns_in_group_mean lag_ns_cross_group_mean last_start_us bands"
