#!/bin/bash
# local 32k fill timeline under engine knobs (experiment build with progress stamps)
mkdir -p gpurun_out
run() {
  env "$@" SA_HIP_LIB=$PWD/build_exp/libsa_prog.so timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 1 > gpurun_out/tlk.json 2>/dev/null || return 1
  python -c "
import json; d=json.load(open('gpurun_out/tlk.json'))
print('$*', d['total_us'], d.get('W'), d.get('cus_used'), d.get('lag_ns_by_checkpoint_in_group'), d.get('lag_ns_by_checkpoint_cross_group'), [r[-1] for r in d['ns_per_step_by_segment_every32']][::2])"
}
run X=0 && run SA_IO_SLEEP=32 && run SA_CHAIN_LDS_KB=120 && run SA_WAVES_PER_GROUP=3 && run SA_WAVES_PER_GROUP=2
