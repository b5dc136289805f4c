# round-5 check 42: strip-step ablations (timing only, results wrong): no plane stores, no merge,
# codes from one address; band and strip step per build, global 32768^2
set -o pipefail
F="total_us ns_per_step_mean clk_per_step_mean"
bash tools/timeline.sh -l "eb nost nomg ccst" -m 32768 -n 32768 -o 0 -f "$F" > /dev/null || exit 1
python3 - <<'PY'
import json
for lib in ("eb", "nost", "nomg", "ccst"):
    d = json.load(open(f"gpurun_out/tl_{lib}_0_32768.json"))
    b = d.get("bands", {})
    print(lib, "strips ns/step", d.get("ns_per_step_mean"), "clk", d.get("clk_per_step_mean"), "end", d.get("last_end_us"),
          "| bands ns/step", b.get("ns_per_step_mean"), "clk", b.get("clk_per_step_mean"), "end", b.get("last_end_us"))
PY
