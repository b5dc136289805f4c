# round-5 check 15: protein (harness dummy requests, BLOSUM50 gap 5) fill-only times with the band
# fill on (default gate) vs off, 65536^2 .. 250000^2, both modes
root=$PWD; bin=$root/sequence-alignment-gpu_amd/bin/sa_benchmarks
mkdir -p gpurun_out/b15_cwd && python tools/score_matrices.py gpurun_out/b15_cwd || exit 1
cd gpurun_out/b15_cwd || exit 1
for rep in 1 2; do for band in def 0; do for t in local global; do
  if [ $band = def ]; then e=""; else e="SA_BAND=0"; fi
  echo "== rep $rep band=$band $t"
  env $e timeout -k 10 120 $bin maxlength $t --sizes 65536x65536,120000x120000,250000x250000 --json | grep '^{' | sed "s/^/band=$band /" || exit 1
done; done; done 2>&1 | tee $root/gpurun_out/b15.log
