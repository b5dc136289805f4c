# round 6: is the band step (43 clk on the last box, 37.7 in round 5's timelines) the round-5 build's
# or this build's? Timelines and bench lines of the round-5 sources (build_exp/libsa_r5.so) and this
# build (build_exp/libsa_cur.so, same experiment flags; product library as "base") on one box; then
# config 5's N = 2 shard with the revised planner (R = 32 when one strip per pair fills the SIMDs)
mkdir -p gpurun_out
: > gpurun_out/timeline.log
for rep in 1 2; do
  SA_TAIL_PAIRS=0 timeout -k 10 300 bash tools/timeline.sh -l "r5 cur base" -f "total_us ns_per_step_mean clk_per_step_mean shader_mhz_mean bands" > /dev/null || exit 1
done
python3 - <<'PY'
import ast
for line in open("gpurun_out/timeline.log"):
    head, d = line.split(" {", 1)
    d = ast.literal_eval("{" + d)
    b = d.get("bands") or {}
    print(head, "strips", d["total_us"], d["ns_per_step_mean"], d["clk_per_step_mean"], "| bands", b.get("last_end_us"), b.get("ns_per_step_mean"), b.get("clk_per_step_mean"), b.get("lag_ns_in_group_mean"), b.get("lag_ns_cross_group_mean"))
PY
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 600 bash tools/ab.sh -l "r5 cur" -w "headline local" -s 20 > /dev/null || exit 1
  SA_TAIL_PAIRS=0 LABEL=base_tail0 timeout -k 10 600 bash tools/ab.sh -w "headline local" -s 20 > /dev/null || exit 1
  LABEL=base_tail timeout -k 10 600 bash tools/ab.sh -w "headline local" -s 20 > /dev/null || exit 1
done
cut -c1-160 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b5_ab.log
timeout -k 10 200 python bench.py --workload batch --shard-of 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6b5_s2.json 2> gpurun_out/r6b5_s2.err || { tail gpurun_out/r6b5_s2.err; exit 1; }
python tools/show_shard.py gpurun_out/r6b5_s2.json
