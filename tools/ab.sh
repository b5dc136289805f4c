#!/bin/bash
# Bench lines of engine builds side by side (GPU box, development): every library x workload runs
# bench.py (no CPU baseline) and prints its key fields (tools/show_bench.py) -> gpurun_out/ab.log.
#   tools/ab.sh [-l "base TAG ..."] [-w "headline local batch"] [-s STEPS] [-- bench.py args]
# LABEL=name replaces the library name in the output lines. TAG = build_exp/libsa_TAG.so (tools/build_exp.sh), base = the product library. Engine knobs in the
# environment pass through (e.g. SA_IO_SLEEP=4, SA_WAVES_PER_GROUP=8, SA_TB_GENERIC=1).
libs=base; wls="headline"; steps=10
while [ $# -gt 0 ]; do
  case $1 in
    -l) libs=$2; shift 2 ;; -w) wls=$2; shift 2 ;; -s) steps=$2; shift 2 ;;
    --) shift; break ;; *) echo "unknown option $1" >&2; exit 2 ;;
  esac
done
mkdir -p gpurun_out
for lib in $libs; do
  L=$PWD/build_exp/libsa_$lib.so; [ "$lib" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  for w in $wls; do
    SA_HIP_LIB=$L timeout -k 10 200 python bench.py --workload $w --steps $steps --warmup 2 --no-cpu-baseline "$@" \
      > gpurun_out/ab_tmp.log 2>&1 || { tail -n 20 gpurun_out/ab_tmp.log; exit 1; }
    echo "== ${LABEL:-$lib} $w $(python tools/show_bench.py gpurun_out/ab_tmp.log)" | tee -a gpurun_out/ab.log
  done
done
