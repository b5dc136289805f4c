# round-4 check 4: A/B of band code-load distance and granule store width (timelines, both modes)
mkdir -p gpurun_out
F="total_us ns_per_step_mean bands"
bash tools/timeline.sh -l "base ah2 g8 ah2g8 base ah2 g8 ah2g8" -m 32768 -o "0 1" -f "$F" > gpurun_out/b4_tl.log 2>&1 || { tail -20 gpurun_out/b4_tl.log; exit 1; }
python3 - <<'PY'
import json, ast
for line in open("gpurun_out/b4_tl.log"):
    head, _, rest = line.partition(" {")
    d = ast.literal_eval("{" + rest)
    b = d.get("bands") or {}
    print(head, "total", d["total_us"], "strip ns/step", d["ns_per_step_mean"], "band ns/step", b.get("ns_per_step_mean"),
          "lag in/cross", b.get("lag_ns_in_group_mean"), b.get("lag_ns_cross_group_mean"), "band end", b.get("last_end_us"))
PY
