# round-5 check 5: band timelines (band step, in-group / cross-group lag) of base0 vs pqx vs pq3, twice
mkdir -p gpurun_out
: > gpurun_out/timeline.log
for rep in 1 2; do
  timeout -k 10 300 bash tools/timeline.sh -l "base0 pqx pq3" -f "total_us bands" > /dev/null || exit 1
done
python3 - <<'PY'
import ast
for line in open("gpurun_out/timeline.log"):
    tag, d = line.split(" {", 1)
    d = ast.literal_eval("{" + d)
    b = d["bands"]
    print(tag, "total", d["total_us"], "band step ns", b["ns_per_step_mean"], "lag in/cross", b["lag_ns_in_group_mean"], b["lag_ns_cross_group_mean"], "last band start/end", b["last_start_us"], b["last_end_us"], "by wave", b["ns_per_step_by_wave_in_group"])
PY
