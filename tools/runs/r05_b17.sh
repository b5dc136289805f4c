# round-5 check 17: one workgroup per CU for the one-wave chain fill (SA_CHAIN_LDS_KB=96 keeps a
# second group off the CU) vs two, vs the band fill; DNA bench lines 65536^2 .. 500000^2 and the
# harness's protein requests
set -o pipefail
root=$PWD
for s in 65536 120000 250000; do
  LABEL=def-$s bash tools/ab.sh -w "headline local" -s 5 -- --size $s || exit 1
  LABEL=band0-$s SA_BAND=0 bash tools/ab.sh -w "headline local" -s 5 -- --size $s || exit 1
  LABEL=band0-1cu-$s SA_BAND=0 SA_CHAIN_LDS_KB=96 bash tools/ab.sh -w "headline local" -s 5 -- --size $s || exit 1
done
LABEL=def-500000 bash tools/ab.sh -w "headline" -s 3 -- --size 500000 || exit 1
LABEL=1cu-500000 SA_CHAIN_LDS_KB=96 bash tools/ab.sh -w "headline" -s 3 -- --size 500000 || exit 1
bin=$root/sequence-alignment-gpu_amd/bin/sa_benchmarks
mkdir -p gpurun_out/b17_cwd && python tools/score_matrices.py gpurun_out/b17_cwd || exit 1
cd gpurun_out/b17_cwd || exit 1
for e in "SA_BAND=1" "SA_BAND=0" "SA_BAND=0 SA_CHAIN_LDS_KB=96"; do for t in local global; do
  env $e timeout -k 10 120 $bin maxlength $t --sizes 65536x65536,120000x120000,250000x250000 --json | grep '^{' | sed "s/^/$e /" || exit 1
done; done 2>&1 | tee -a $root/gpurun_out/ab.log
