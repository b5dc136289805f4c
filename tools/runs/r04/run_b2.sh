# round-4 development check 2: GPU suite, band timelines (probe on/off, bands alone), headline bench, rocprof
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b2_tests.log 2>&1 || { tail -n 40 gpurun_out/b2_tests.log; exit 1; }
tail -n 2 gpurun_out/b2_tests.log
F="total_us ns_per_step_mean lag_ns_in_group_mean bands"
bash tools/timeline.sh -l "base nostrips nostripsconst nostripsnodrain" -m 32768 -o "0 1" -f "$F" || exit 1
SA_IO_PROBE=0 bash tools/timeline.sh -l base -m 32768 -o "0 1" -f "$F" || exit 1
for w in headline local; do
  timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b2_$w.json 2> gpurun_out/b2_$w.err || { tail -n 20 gpurun_out/b2_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/b2_$w.json
  SA_TB_STAGER=0 timeout -k 10 200 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b2_${w}_nostager.json 2> gpurun_out/b2_$w.err || { tail -n 20 gpurun_out/b2_$w.err; exit 1; }
  python tools/show_bench.py gpurun_out/b2_${w}_nostager.json
done
bash tools/profile_all.sh b2
