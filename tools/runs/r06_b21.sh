# round 6: the encode kernel resets the fill's control word (no memset launch per fill; bad_input
# epoch-tagged): the full GPU suite, then the bench lines against the previous build
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6b21_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b21_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b21_tests.log
: > gpurun_out/ab.log
for rep in 1 2 3; do
  timeout -k 10 600 bash tools/ab.sh -l "base prevctl" -w "headline dna8k protein4k" -s 20 > /dev/null || exit 1
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b21_ab.log
