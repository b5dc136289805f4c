# round 6: ADVICE fixes (local M with STOP from fetch_directions, walker bound -> status, compact strip
# tables, long local table-traceback test), then the config-5 shard sweep (rank 0's shard of N on one
# GPU) x rows per lane (0 = planner)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_tb_tables.py tests/test_gpu_parity.py tests/test_band_fill.py > gpurun_out/r6b1_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b1_tests.log; exit 1; }
tail -n 2 gpurun_out/r6b1_tests.log
for N in 1 2 4 8; do
  for R in 0 16 8 4; do
    timeout -k 10 200 python bench.py --workload batch --shard-of $N --rows-per-lane $R --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/r6b1_s${N}_r${R}.json 2> gpurun_out/r6b1_s${N}_r${R}.err || { tail -n 20 gpurun_out/r6b1_s${N}_r${R}.err; exit 1; }
    python - gpurun_out/r6b1_s${N}_r${R}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["config"]["rows_per_lane"], d["config"]["strips_per_gpu"], "step", d["ms_per_step"], "fill", d["fill_ms_per_launch"]["median"], "tb", d["e2e_ms"]["traceback"], "pair0", d["sample_result"]["pair0_score"])
PY
  done
done
