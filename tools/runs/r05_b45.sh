# round-5 check 45: lone strip (m = 64), a fed strip (m = 128: strip 1 reads strip 0's ring), a
# group of four (m = 256) and the full chain: per-strip step in shader clocks, product build
set -o pipefail
F="total_us ns_per_step_mean clk_per_step_mean ns_per_step_by_strip slow_paths_mean_per_strip"
bash tools/timeline.sh -l "base" -m "64 128 256 1024" -o "0 1" -f "$F" || exit 1
