# round-4 check 8: traceback phase split with the stager (walk-timing build), then the harness modes
mkdir -p gpurun_out
for st in 1 0; do
  for mode in 0 1; do
    SA_TB_STAGER=$st SA_HIP_LIB=$PWD/build_exp/libsa_wt.so timeout -k 10 120 python tools/tb_timing.py --mode $mode > gpurun_out/b8_tb_${st}_$mode.json 2> gpurun_out/b8_tb.err || { tail -20 gpurun_out/b8_tb.err; exit 1; }
    echo "stager=$st $(cat gpurun_out/b8_tb_${st}_$mode.json)"
  done
done
bash tools/harness.sh b8 > /dev/null || exit 1
cat gpurun_out/b8_harness.jsonl
