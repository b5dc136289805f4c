mkdir -p gpurun_out; : > gpurun_out/tlp.log
for c in "64 1" "64 4" "64 16" "64 1024" "128 1" "128 4"; do set -- $c
  echo "== m=$1 pairs=$2" >> gpurun_out/tlp.log
  timeout -k 10 60 python tools/timeline.py --n 32768 --m $1 --pairs $2 --waves 4 2>&1 | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('total_us','ns_per_step_mean','ns_per_step_min','ns_per_step_max','clk_per_step_mean','cus_used','max_strips_on_one_simd_concurrently')})" >> gpurun_out/tlp.log || exit 1
done
cat gpurun_out/tlp.log
