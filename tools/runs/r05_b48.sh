# round-5 check 48: strip start slack (SA_EXP_STRIP_SLACK: in-group consumers start 64 / 192 columns
# later than they must) against the experiment build: timelines, then bench lines twice
set -o pipefail
F="total_us ns_per_step_mean clk_per_step_mean"
bash tools/timeline.sh -l "eb sl64 sl192" -m "32768" -o "0 1" -f "$F" || exit 1
rm -f gpurun_out/ab.log
timeout -k 10 900 bash tools/ab.sh -l "eb sl64 sl192 eb sl64 sl192" -w "headline local dna8k" -s 10 || exit 1
