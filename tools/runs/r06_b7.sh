# round 6: tail strip groups as their own kernel instance (fill_kernel<..., VG>; the default band
# kernels are the round-5 code again): tail tests, then a same-box A/B and timelines of groups of 4
# (SA_TAIL_PAIRS=0), pairs only (SA_TAIL_LONE=0) and pairs + lone strips (default)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_band_fill.py > gpurun_out/r6b7_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b7_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b7_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  SA_TAIL_PAIRS=0 LABEL=tail0 timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k protein4k" -s 20 > /dev/null || exit 1
  SA_TAIL_LONE=0 LABEL=pairs timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k protein4k" -s 20 > /dev/null || exit 1
  LABEL=lone timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k protein4k" -s 20 > /dev/null || exit 1
done
cut -c1-170 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b7_ab.log
for v in "0 0" "1 0" "1 -1"; do
  set -- $v
  tag=tail$1_$2
  if [ "$2" = "-1" ]; then env_lone=""; else env_lone="SA_TAIL_LONE=$2"; fi
  for mode in 0 1; do
    env SA_TAIL_PAIRS=$1 $env_lone timeout -k 10 120 python tools/timeline.py --n 32768 --m 32768 --mode $mode > gpurun_out/r6b7_tl_${tag}_$mode.json 2> gpurun_out/r6b7_tl_err.log || { cat gpurun_out/r6b7_tl_err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for tp in ("tail0_0", "tail1_0", "tail1_-1"):
    for mode in (0, 1):
        d = json.load(open(f"gpurun_out/r6b7_tl_{tp}_{mode}.json"))
        b = d.get("bands", {})
        print(tp, "mode", mode, "strips end", d["last_end_us"], "ns/step", d["ns_per_step_mean"], "| bands end", b.get("last_end_us"), "ns/step", b.get("ns_per_step_mean"))
        print("   strip ns/step by strip", d.get("ns_per_step_by_strip"))
PY
