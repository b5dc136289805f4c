#!/bin/bash
# Hand-off timing ablations (development): timelines of build_exp/libsa_<tag>.so builds whose
# results are wrong by design (SA_ABL), next to the product library ("base").
mkdir -p gpurun_out
log=gpurun_out/tla.log
: > $log
for v in "$@"; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  for m in 64 256 32768; do
    echo "== $v m=$m" >> $log
    SA_HANDOFF_TIMEOUT_S=0.05 SA_HIP_LIB=$L timeout -k 10 60 python tools/timeline.py --n 32768 --m $m --waves 4 2>&1 | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('total_us','clk_per_step_mean','lag_ns_in_group_mean','lag_ns_cross_group_mean','ns_per_step_by_strip')})" >> $log || exit 1
  done
done
cat $log
