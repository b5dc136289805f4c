# round-5 check 18: chain_solo build; band tests, then band vs one-wave (one workgroup per CU) around
# the crossover, DNA bench lines and the harness's protein requests (warm, throughput mode)
set -o pipefail
root=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_band_fill.py > gpurun_out/b18_tests.log 2>&1 || { tail -30 gpurun_out/b18_tests.log; exit 1; }
tail -2 gpurun_out/b18_tests.log
for s in 65536 81920 98304 120000; do
  LABEL=band1-$s SA_BAND=1 bash tools/ab.sh -w "headline local" -s 5 -- --size $s || exit 1
  LABEL=band0-$s SA_BAND=0 bash tools/ab.sh -w "headline local" -s 5 -- --size $s || exit 1
done
bin=$root/sequence-alignment-gpu_amd/bin/sa_benchmarks
mkdir -p gpurun_out/b18_cwd && python tools/score_matrices.py gpurun_out/b18_cwd || exit 1
cd gpurun_out/b18_cwd || exit 1
for e in "SA_BAND=1" "SA_BAND=0"; do for t in local global; do
  env $e timeout -k 10 150 $bin throughput $t --repeats 2 --sizes 32768x32768,49152x49152,65536x65536,98304x98304 --json | grep '^{' | sed "s/^/$e /" || exit 1
done; done 2>&1 | tee -a $root/gpurun_out/ab.log
