#!/bin/bash
# local 32k slow phase: progress-stamped timelines of ablation builds (prog = base, nostore = no
# direction-plane stores, codesconst = text-code loads from a fixed 64-byte window; results wrong)
mkdir -p gpurun_out
for v in ${VARIANTS:-prog nostore codesconst}; do
  SA_HIP_LIB=$PWD/build_exp/libsa_$v.so timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 1 > gpurun_out/tla.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/tla.json'))
print('$v', d['total_us'], [r[-1] for r in d['ns_per_step_by_segment_every32']][::2], d['ns_per_step_by_segment_every32'][8])"
done
