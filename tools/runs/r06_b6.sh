# round 6: bisect the band-step regression (43 vs 37.7 clk): the fill_r1 unit of commits 8acc629 (r5),
# 309f954 (pair chains), b6584b3 (strip group table), 3bc53cf (pair priority), ff2be44 (head) over
# this build's other units, timelines on one box; then R = 4 pair chains (tests, shard 4 / 8 sweep)
mkdir -p gpurun_out
: > gpurun_out/timeline.log
for rep in 1 2; do
  SA_TAIL_PAIRS=0 timeout -k 10 400 bash tools/timeline.sh -l "b_r5 b_p1 b_p2 b_p3 b_cur" -f "total_us ns_per_step_mean clk_per_step_mean bands" > /dev/null || exit 1
done
python3 - <<'PY'
import ast
for line in open("gpurun_out/timeline.log"):
    head, d = line.split(" {", 1)
    d = ast.literal_eval("{" + d)
    b = d.get("bands") or {}
    print(head, "strips", d["total_us"], d["ns_per_step_mean"], d["clk_per_step_mean"], "| bands", b.get("last_end_us"), b.get("ns_per_step_mean"), b.get("clk_per_step_mean"), b.get("lag_ns_in_group_mean"), b.get("lag_ns_cross_group_mean"))
PY
cp gpurun_out/timeline.log gpurun_out/r6b6_timeline.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_batch_golden.py -k "pair_packed or shard or config5" > gpurun_out/r6b6_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b6_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b6_tests.log
for N in 4 8; do
  for CR in 8 4; do
    SA_PAIR_CHAIN_R=$CR timeout -k 10 200 python bench.py --workload batch --shard-of $N --steps 10 --warmup 3 --no-cpu-baseline \
      > gpurun_out/r6b6_s${N}_c${CR}.json 2> gpurun_out/r6b6_s${N}_c${CR}.err || { tail -n 20 gpurun_out/r6b6_s${N}_c${CR}.err; exit 1; }
    python tools/show_shard.py gpurun_out/r6b6_s${N}_c${CR}.json
  done
done
