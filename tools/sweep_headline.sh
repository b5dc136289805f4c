mkdir -p gpurun_out; : > gpurun_out/swh.log
for c in "1 4" "2 4" "4 4" "1 3" "1 2"; do set -- $c
  echo "== R=$1 W=$2" >> gpurun_out/swh.log
  SA_WAVES_PER_GROUP=$2 timeout -k 10 120 python bench.py --workload headline --rows-per-lane $1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/swh_tmp.log 2>&1 || { cat gpurun_out/swh_tmp.log; exit 1; }
  python tools/show_bench.py gpurun_out/swh_tmp.log >> gpurun_out/swh.log
done
cat gpurun_out/swh.log
