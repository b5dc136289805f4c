# round-5 check 16: one-wave fill (SA_BAND=0) timelines at 120000^2, global vs local, protein and DNA
F="total_us ns_per_step_mean clk_per_step_mean lag_ns_in_group_mean lag_ns_cross_group_mean lag_ns_p90 max_strips_on_one_simd_concurrently shader_mhz_mean"
SA_BAND=0 bash tools/timeline.sh -m 120000 -n 120000 -o "0 1" -f "$F" -- --protein &&
SA_BAND=0 bash tools/timeline.sh -m 120000 -n 120000 -o "0 1" -f "$F"
