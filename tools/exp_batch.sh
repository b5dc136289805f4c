# fill-only timing of the batch workload for experiment builds in build_exp/
for v in "$@"; do
  L=$PWD/build_exp/libsa_$v.so; [ "$v" = base ] && L=$PWD/sequence-alignment-gpu_amd/lib/libsa_hip.so
  echo "== $v" >> gpurun_out/expb.log
  SA_HIP_LIB=$L timeout -k 10 120 python bench.py --workload batch --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/expb.log 2>&1 || exit 1
  SA_HIP_LIB=$L timeout -k 10 120 python bench.py --workload headline --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/expb.log 2>&1 || exit 1
done
