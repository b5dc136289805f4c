# round-5 check 38: band-fill timelines, global and local 32768^2 (band step / lag, strip step)
set -o pipefail
F="total_us ns_per_step_mean clk_per_step_mean lag_ns_in_group_mean lag_ns_cross_group_mean shader_mhz_mean"
bash tools/timeline.sh -m 32768 -n 32768 -o "0 1" -f "$F" || exit 1
python3 - <<'PY'
import json
for mode in (0, 1):
    d = json.load(open(f"gpurun_out/tl_base_{mode}_32768.json"))
    b = d.get("bands", {})
    print("mode", mode, "bands", {k: b.get(k) for k in ("total_us", "ns_per_step_mean", "clk_per_step_mean", "lag_ns_in_group_mean", "lag_ns_cross_group_mean", "last_start_us", "last_end_us", "ns_per_step_by_wave_in_group", "simd_by_wave_in_group")})
    print("mode", mode, "strips", {k: d.get(k) for k in ("total_us", "ns_per_step_mean", "clk_per_step_mean", "last_start_us", "last_end_us", "ns_per_step_by_wave_in_group")})
PY
