#!/bin/bash
# Fill timing of experiment builds (build_exp/libsa_<tag>.so, "base" = the product library):
# headline / local / batch bench lines and a lone-strip + full-chain timeline per build.
mkdir -p gpurun_out
log=gpurun_out/expc.log
: > $log
for v in "$@"; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  for w in headline local batch; do
    echo "== $v $w" >> $log
    SA_HIP_LIB=$L timeout -k 10 120 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/expc_tmp.log 2>&1 || { cat gpurun_out/expc_tmp.log; exit 1; }
    python tools/show_bench.py gpurun_out/expc_tmp.log >> $log
  done
  for c in "64 4" "32768 4"; do set -- $c
    echo "== $v timeline m=$1" >> $log
    SA_HIP_LIB=$L timeout -k 10 60 python tools/timeline.py --n 32768 --m $1 --waves $2 2>&1 | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('total_us','ns_per_step_mean','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean')})" >> $log || exit 1
  done
done
cat $log
