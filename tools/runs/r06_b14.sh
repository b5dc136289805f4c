# round 6: copy-0 profile reads (kArr8A) for DNA too (SA_ALIGN=2, parity of the band tests first) and
# with the global bands' code touch (build_exp/libsa_atouch.so, SA_EXP_ALIGN_TOUCH): same-box A/Bs
mkdir -p gpurun_out
SA_ALIGN=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_band_fill.py tests/test_gpu_parity.py > gpurun_out/r6b14_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b14_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b14_tests.log
: > gpurun_out/ab.log
for rep in 1 2 3; do
  timeout -k 10 600 bash tools/ab.sh -l "base atouch" -w "protein4k" -s 20 > /dev/null || exit 1
done
for rep in 1 2; do
  timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k" -s 20 > /dev/null || exit 1
  SA_ALIGN=2 LABEL=align2 timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k" -s 20 > /dev/null || exit 1
  SA_ALIGN=2 LABEL=align2touch timeout -k 10 600 bash tools/ab.sh -l atouch -w "headline dna8k" -s 20 > /dev/null || exit 1
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b14_ab.log
