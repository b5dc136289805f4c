# round-5 check 46: strip feed ablations (timing only, results wrong): fnr = no feed read (a value that
# passes the tag check), fnc = the read and its wait but no check; eb = the experiment build unchanged
set -o pipefail
F="total_us ns_per_step_mean clk_per_step_mean ns_per_step_by_strip"
bash tools/timeline.sh -l "eb fnr fnc" -m "128 32768" -o "0 1" -f "$F" || exit 1
