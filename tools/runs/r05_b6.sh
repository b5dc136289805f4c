# round-5 check 6: XCD-local band chain (SA_BAND_XCD=1: per-XCD band queues, near granules through
# the XCD's L2) -- band / parity / edge GPU tests with it on, then a same-box A/B of the knob off / on
# (one library), then band timelines off / on
mkdir -p gpurun_out
SA_BAND_XCD=1 timeout -k 10 500 python -u -m pytest tests/test_band_fill.py tests/test_gpu_parity.py tests/test_edge_cases.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b6_tests.log 2>&1 || { tail -n 30 gpurun_out/r5b6_tests.log; exit 1; }
tail -n 1 gpurun_out/r5b6_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  for x in 0 1; do
    LABEL=xcd$x SA_BAND_XCD=$x timeout -k 10 400 bash tools/ab.sh -l base -w "headline local dna8k" -s 20 > /dev/null || exit 1
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
    print(tag, "total", d["total_us"], "band step ns", b["ns_per_step_mean"], "lag in/cross", b["lag_ns_in_group_mean"], b["lag_ns_cross_group_mean"], "last band start/end", b["last_start_us"], b["last_end_us"])
PY
