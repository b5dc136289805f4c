# round-5 check 39: strip waves at priority 2 (SA_EXP_STRIP_PRIO) vs the same build without:
# timelines (band / strip step) and bench lines, same box
set -o pipefail
F="total_us ns_per_step_mean clk_per_step_mean lag_ns_in_group_mean"
bash tools/timeline.sh -l "eb sprio" -m 32768 -n 32768 -o "0 1" -f "$F" || exit 1
for rep in 1 2; do
  bash tools/ab.sh -l "eb sprio" -w "headline local dna8k" || exit 1
done
