#!/bin/bash
# Per-strip fill timelines (tools/timeline.py) over engine builds x chain lengths x modes: one
# summary line per run on stdout and in gpurun_out/timeline.log; full JSON in
# gpurun_out/tl_<lib>_<mode>_<m>.json. Development tool, run on the GPU box.
#   tools/timeline.sh [-l "base TAG ..."] [-m "64 256 32768"] [-o "0 1"] [-n N] [-f "field ..."] [-- timeline.py args]
# TAG = build_exp/libsa_TAG.so (tools/build_exp.sh), base = the product library. Engine knobs in the
# environment (SA_IO_SLEEP, SA_WAVES_PER_GROUP, SA_HANDOFF_TIMEOUT_S ...) pass through.
# Examples: lone strip vs chain   tools/timeline.sh -m "64 256 32768"
#           A/B of builds         tools/timeline.sh -l "base pf14" -o "0 1"
#           waves per group       SA_WAVES_PER_GROUP=8 tools/timeline.sh -- --waves 8
#           concurrent chains     tools/timeline.sh -m 2048 -- --pairs 16
libs=base; ms="32768"; modes="0"; n=32768
fields="total_us ns_per_step_mean clk_per_step_mean lag_ns_in_group_mean lag_ns_cross_group_mean shader_mhz_mean"
while [ $# -gt 0 ]; do
  case $1 in
    -l) libs=$2; shift 2 ;; -m) ms=$2; shift 2 ;; -o) modes=$2; shift 2 ;; -n) n=$2; shift 2 ;;
    -f) fields=$2; shift 2 ;; --) shift; break ;; *) echo "unknown option $1" >&2; exit 2 ;;
  esac
done
mkdir -p gpurun_out
for lib in $libs; do
  L=$PWD/build_exp/libsa_$lib.so; [ "$lib" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  for mode in $modes; do for m in $ms; do
    out=gpurun_out/tl_${lib}_${mode}_$m.json
    SA_HIP_LIB=$L timeout -k 10 60 python tools/timeline.py --n $n --m $m --mode $mode "$@" > $out 2> gpurun_out/tl_err.log ||
      { cat gpurun_out/tl_err.log; exit 1; }
    python3 - "$out" "$lib mode=$mode m=$m" $fields <<'PY' | tee -a gpurun_out/timeline.log
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: d.get(k) for k in sys.argv[3:]})
PY
  done; done
done
