# round-4 check 5: GPU suite; same-box A/B of the product against round 4's first band build (r4b1)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b5_tests.log 2>&1 || { tail -n 40 gpurun_out/b5_tests.log; exit 1; }
tail -n 2 gpurun_out/b5_tests.log
F="total_us ns_per_step_mean bands"
bash tools/timeline.sh -l "base r4b1 base r4b1 base r4b1" -m 32768 -o "0 1" -f "$F" > gpurun_out/b5_tl.log 2>&1 || { tail -20 gpurun_out/b5_tl.log; exit 1; }
python3 - <<'PY'
import ast
for line in open("gpurun_out/b5_tl.log"):
    head, _, rest = line.partition(" {")
    d = ast.literal_eval("{" + rest)
    b = d.get("bands") or {}
    print(head, "total", d["total_us"], "strip ns/step", d["ns_per_step_mean"], "band ns/step", b.get("ns_per_step_mean"),
          "lag in/cross", b.get("lag_ns_in_group_mean"), b.get("lag_ns_cross_group_mean"), "band end", b.get("last_end_us"))
PY
