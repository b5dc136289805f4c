# round 6: ADVICE fixes + pair-packed chains (fill_pair_chain_kernel) + planner sized to the GPU:
# the touched GPU tests, then the config-5 shard sweep (rank 0's shard of N on one GPU) x rows per
# lane (0 = planner; 16/8/4 forced: pair chains for 16/8, the one-wave chained fill for 4)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_batch_golden.py tests/test_tb_tables.py tests/test_band_fill.py tests/test_edge_cases.py > gpurun_out/r6b2_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b2_tests.log; exit 1; }
tail -n 2 gpurun_out/r6b2_tests.log
for N in 1 2 4 8; do
  for R in 0 32 16 8; do
    timeout -k 10 200 python bench.py --workload batch --shard-of $N --rows-per-lane $R --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/r6b2_s${N}_r${R}.json 2> gpurun_out/r6b2_s${N}_r${R}.err || { tail -n 20 gpurun_out/r6b2_s${N}_r${R}.err; exit 1; }
    python tools/show_shard.py gpurun_out/r6b2_s${N}_r${R}.json
  done
done
