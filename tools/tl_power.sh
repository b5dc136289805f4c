#!/bin/bash
# Is the late slowdown of long local fills time-based (power / clock) or chain-based? 16 short chains
# (m = 2048) over 65536 columns vs the 32k chain; ns and shader clocks per step per 4096-column segment
mkdir -p gpurun_out
run() {
  SA_HIP_LIB=$PWD/build_exp/libsa_prog.so timeout -k 10 60 python tools/timeline.py --mode 1 "$@" > gpurun_out/tlpw.json 2>/dev/null || return 1
  python -c "
import json; d=json.load(open('gpurun_out/tlpw.json'))
print('$*', d['total_us'], 'ns', d['ns_per_step_by_segment_every32'][-1], 'clk', d['clk_per_step_by_segment_every32'][-1], d['clk_per_step_by_segment_every32'][0])"
}
run --n 65536 --m 2048 --pairs 16 && run --n 32768 --m 32768 && run --n 65536 --m 2048 --pairs 4
