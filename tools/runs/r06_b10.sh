# round 6: what slows the protein bands (51 clk per step against 38.6 for DNA): the same BLOSUM50 band
# kernel with the sequences drawn from 20 / 8 / 4 / 1 letters (fewer distinct text-profile rows per
# wave load)
mkdir -p gpurun_out
for L in 20 8 4 1; do
  timeout -k 10 120 python tools/timeline.py --n 4096 --m 4096 --protein --letters $L --mode 0 > gpurun_out/r6b10_tl_p$L.json 2> gpurun_out/r6b10_tl_err.log || { cat gpurun_out/r6b10_tl_err.log; exit 1; }
done
python3 - <<'PY'
import json
for L in (20, 8, 4, 1):
    d = json.load(open(f"gpurun_out/r6b10_tl_p{L}.json"))
    b = d.get("bands", {})
    print("letters", L, "strips end", d["last_end_us"], "clk", d["clk_per_step_mean"], "| bands end", b.get("last_end_us"), "clk", b.get("clk_per_step_mean"),
          "lag in/cross", b.get("lag_ns_in_group_mean"), b.get("lag_ns_cross_group_mean"))
PY
