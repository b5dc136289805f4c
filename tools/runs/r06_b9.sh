# round 6: the N-rank bench path on one GPU (two gloo ranks on device 0), protein / 8192^2 timelines
# (where configs 2 and 4 spend their time), and the reference harness modes
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_distributed.py > gpurun_out/r6b9_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b9_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b9_tests.log
for spec in "--n 8192 --m 8192:dna8k" "--n 4096 --m 4096 --protein:protein4k"; do
  args=${spec%%:*}; tag=${spec##*:}
  timeout -k 10 120 python tools/timeline.py $args --mode 0 > gpurun_out/r6b9_tl_$tag.json 2> gpurun_out/r6b9_tl_err.log || { cat gpurun_out/r6b9_tl_err.log; exit 1; }
done
python3 - <<'PY'
import json
for tag in ("dna8k", "protein4k"):
    d = json.load(open(f"gpurun_out/r6b9_tl_{tag}.json"))
    b = d.get("bands", {})
    print(tag, "strips end", d["last_end_us"], "first fed", d["first_fed_us"], "ns/step", d["ns_per_step_mean"], "clk", d["clk_per_step_mean"],
          "| bands end", b.get("last_end_us"), "ns/step", b.get("ns_per_step_mean"), "clk", b.get("clk_per_step_mean"),
          "lag in/cross", b.get("lag_ns_in_group_mean"), b.get("lag_ns_cross_group_mean"), "strip lag", d.get("lag_ns_in_group_mean"))
PY
timeout -k 10 1500 bash tools/harness.sh r6b9 > gpurun_out/r6b9_harness_out.log 2>&1 || { tail -n 20 gpurun_out/r6b9_harness_out.log; exit 1; }
tail -n 12 gpurun_out/r6b9_harness_out.log
