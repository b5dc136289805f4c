# round 6: local protein with and without the copy-0 profile reads (SA_ALIGN=1 / 0), the reference
# harness's throughput local and maxlength local modes (its dummy protein requests), same box
mkdir -p gpurun_out/r6b16_cwd
python tools/score_matrices.py gpurun_out/r6b16_cwd || exit 1
bin=$PWD/sequence-alignment-gpu_amd/bin/sa_benchmarks
out=$PWD/gpurun_out/r6b16.log
: > $out
cd gpurun_out/r6b16_cwd || exit 1
for rep in 1 2; do
  for al in 1 0; do
    echo "== SA_ALIGN=$al throughput local" >> $out
    SA_ALIGN=$al timeout -k 10 240 $bin throughput local --repeats 3 --sizes 16384x16384,32768x32768,65536x65536 --json >> $out 2>&1 || exit 1
    echo "== SA_ALIGN=$al throughput global" >> $out
    SA_ALIGN=$al timeout -k 10 240 $bin throughput global --repeats 3 --sizes 16384x16384,32768x32768,65536x65536 --json >> $out 2>&1 || exit 1
    echo "== SA_ALIGN=$al maxlength local" >> $out
    SA_ALIGN=$al timeout -k 10 240 $bin maxlength local --json >> $out 2>&1 || exit 1
  done
done
grep "==\|\"rows\": 32768\|\"rows\": 65536\|maxlength" $out | cut -c1-160
