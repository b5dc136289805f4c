# round-4 check 3: band code loads four bodies ahead
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b3_tests.log 2>&1 || { tail -n 40 gpurun_out/b3_tests.log; exit 1; }
tail -n 2 gpurun_out/b3_tests.log
bash tools/timeline.sh -l base -m 32768 -o "0 1" -f "total_us ns_per_step_mean bands" || exit 1
for w in headline local dna8k protein4k; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b3_$w.json 2> gpurun_out/b3_$w.err || { tail -n 20 gpurun_out/b3_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/b3_$w.json
done
