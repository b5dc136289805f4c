# round-5 check 27: table traceback at large sizes (e2e traceback times, fallbacks show as the old
# sequential times), and the harness latency lines
set -o pipefail
for s in 65536 120000 250000 500000; do
  LABEL=tb-$s bash tools/ab.sh -w "headline local" -s 3 -- --size $s || exit 1
done
bin=$PWD/sequence-alignment-gpu_amd/bin/sa_benchmarks
mkdir -p gpurun_out/b27_cwd && python tools/score_matrices.py gpurun_out/b27_cwd || exit 1
cd gpurun_out/b27_cwd || exit 1
for t in global local; do
  timeout -k 10 200 $bin latency $t --repeats 2 --json | grep '^{' || exit 1
done 2>&1 | tee -a ../ab.log
