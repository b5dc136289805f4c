# round-5 check 7: same-box A/B of the round-start build (base0) against HEAD + XCD knob off / on, and
# band timelines with the XCD split of the cross-group lag
mkdir -p gpurun_out
: > gpurun_out/ab.log
for rep in 1 2; do
  LABEL=base0 timeout -k 10 400 bash tools/ab.sh -l base0 -w "headline" -s 20 > /dev/null || exit 1
  for x in 0 1; do
    LABEL=xcd$x SA_BAND_XCD=$x timeout -k 10 400 bash tools/ab.sh -l base -w "headline" -s 20 > /dev/null || exit 1
  done
done
cut -c1-110 gpurun_out/ab.log
: > gpurun_out/timeline.log
for x in 0 1; do
  SA_BAND_XCD=$x timeout -k 10 200 bash tools/timeline.sh -l base -f "total_us bands" > /dev/null || exit 1
done
python3 - <<'PY'
import ast
for line in open("gpurun_out/timeline.log"):
    tag, d = line.split(" {", 1)
    d = ast.literal_eval("{" + d)
    b = d["bands"]
    print(tag, "total", d["total_us"], "step", b["ns_per_step_mean"], "lag in/cross", b["lag_ns_in_group_mean"], b["lag_ns_cross_group_mean"], "cross same/other xcd", b["lag_ns_cross_same_xcd"], b["lag_ns_cross_other_xcd"], b["cross_same_xcd_count"], "xcc", b["xcc_by_record_first32"])
PY
