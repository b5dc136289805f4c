#!/bin/bash
# progress stamps (experiment build build_exp/libsa_prog.so): pace per 4096-column segment along the
# chain, local 32k with the blast scores (long alignment, large H) and with +1/-3 (H stays small)
set -e
mkdir -p gpurun_out
for sc in blast; do
  SA_HIP_LIB=$PWD/build_exp/libsa_prog.so timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 1 --score $sc > gpurun_out/tlprog_$sc.json 2>/dev/null
  python -c "
import json; d=json.load(open('gpurun_out/tlprog_$sc.json'))
print('$sc', {k: d.get(k) for k in ('total_us','clk_per_step_mean','ns_per_step_by_segment_every32','lag_ns_by_checkpoint_in_group','lag_ns_by_checkpoint_cross_group')})"
done
