mkdir -p gpurun_out; : > gpurun_out/la.log
for v in base la2 base la2; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  echo "== $v" >> gpurun_out/la.log
  SA_HIP_LIB=$L timeout -k 10 120 python bench.py --workload local --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/la_tmp.log 2>&1 || exit 1
  python tools/show_bench.py gpurun_out/la_tmp.log >> gpurun_out/la.log
done
cat gpurun_out/la.log
