# round 6: band fill with tail strip groups of 2 (SA_TAIL_PAIRS, default on): band / parity tests, then a
# same-box A/B against groups of 4 everywhere (SA_TAIL_PAIRS=0), three repetitions, and timelines
mkdir -p gpurun_out
# (the band / parity tests run in r06_b2.sh, which r06_b4.sh runs first)
: > gpurun_out/ab.log
for rep in 1 2; do
  SA_TAIL_PAIRS=0 LABEL=tail0 timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k protein4k" -s 20 > /dev/null || exit 1
  SA_TAIL_LONE=0 LABEL=pairs timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k protein4k" -s 20 > /dev/null || exit 1
  LABEL=lone timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k protein4k" -s 20 > /dev/null || exit 1
done
cut -c1-160 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b3_ab_tail.log
for v in "0 0" "1 0" "1 -1"; do
  set -- $v
  tag=tail$1_$2
  if [ "$2" = "-1" ]; then env_lone=""; else env_lone="SA_TAIL_LONE=$2"; fi
  env SA_TAIL_PAIRS=$1 $env_lone timeout -k 10 120 python tools/timeline.py --n 32768 --m 32768 --mode 0 > gpurun_out/r6b3_tl_$tag.json 2> gpurun_out/r6b3_tl_err.log || { cat gpurun_out/r6b3_tl_err.log; exit 1; }
done
python3 - <<'PY'
import json
for tp in ("tail0_0", "tail1_0", "tail1_-1"):
    d = json.load(open(f"gpurun_out/r6b3_tl_{tp}.json"))
    b = d.get("bands", {})
    print("tail", tp, "strips", {k: d.get(k) for k in ("total_us", "last_start_us", "last_end_us", "ns_per_step_mean", "cus_used")},
          "bands", {k: b.get(k) for k in ("last_start_us", "last_end_us", "ns_per_step_mean", "lag_ns_in_group_mean", "lag_ns_cross_group_mean")})
    print("   strip ns/step by strip", d.get("ns_per_step_by_strip"))
PY
# the pipelined batch step with the pair-packed fill at issue priority 2 (SA_PAIR_PRIO) vs default
: > gpurun_out/ab.log
for rep in 1 2 3; do
  for pp in 0 1; do
    SA_PAIR_PRIO=$pp LABEL=prio$pp timeout -k 10 600 bash tools/ab.sh -w "batch" -s 20 > /dev/null || exit 1
  done
done
cut -c1-200 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b3_ab_prio.log
