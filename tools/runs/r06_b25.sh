# round 6: single-pair plans reset their control word in the encode kernel (no memset launch), plans
# of several pairs keep the launch: the full GPU suite, then bench lines against the product build
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6b25_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b25_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b25_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 900 bash tools/ab.sh -l "base prod" -w "headline dna8k protein4k batch" -s 20 > /dev/null || exit 1
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b25_ab.log
