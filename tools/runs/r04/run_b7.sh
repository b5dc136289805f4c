# round-4 check 7: band feed-read step (pf12 / pf13 vs 10) and I/O wave idle sleep (1 / 2 vs 4), global 32768^2
mkdir -p gpurun_out
F="total_us ns_per_step_mean bands"
{ bash tools/timeline.sh -l "base pf12 pf13" -m 32768 -o 0 -f "$F" &&
  SA_IO_SLEEP=1 bash tools/timeline.sh -l base -m 32768 -o 0 -f "$F" && SA_IO_SLEEP=2 bash tools/timeline.sh -l base -m 32768 -o 0 -f "$F" &&
  bash tools/timeline.sh -l "base pf12 pf13" -m 32768 -o 0 -f "$F" &&
  SA_IO_SLEEP=1 bash tools/timeline.sh -l base -m 32768 -o 0 -f "$F" && SA_IO_SLEEP=2 bash tools/timeline.sh -l base -m 32768 -o 0 -f "$F"; } > gpurun_out/b7_tl.log 2>&1 || { tail -20 gpurun_out/b7_tl.log; exit 1; }
python3 - <<'PY'
import ast
for line in open("gpurun_out/b7_tl.log"):
    head, _, rest = line.partition(" {")
    d = ast.literal_eval("{" + rest)
    b = d.get("bands") or {}
    print(head, "total", d["total_us"], "strip ns/step", d["ns_per_step_mean"], "band ns/step", b.get("ns_per_step_mean"),
          "lag in/cross", b.get("lag_ns_in_group_mean"), b.get("lag_ns_cross_group_mean"), "band end", b.get("last_end_us"))
PY
