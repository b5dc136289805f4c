# round-5 check 47: feed-miss counters of the strips (SA_EXP_PROGRESS build), global and local 32768^2
set -o pipefail
F="total_us ns_per_step_mean slow_paths_mean_per_strip feed_slow_by_wave_in_group feed_slow_past_4096_by_wave_in_group feed_spins_past_4096_by_wave_in_group io_ahead_us_every8groups"
bash tools/timeline.sh -l "prog" -m "32768" -o "0 1" -f "$F" || exit 1
