# round-5 check 9: band fill with persistent workers past resident capacity -- the forced-CU-cap
# band test and the whole band suite, then bench lines at 65536^2 and 120000^2 (band fill now) against
# the one-wave fill (SA_BAND=0), and the 32768^2 headline (unchanged path)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_band_fill.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b9_tests.log 2>&1 || { tail -n 30 gpurun_out/r5b9_tests.log; exit 1; }
tail -n 1 gpurun_out/r5b9_tests.log
: > gpurun_out/ab.log
for sz in 65536 120000; do
  for b in 1 0; do
    LABEL=band$b SA_BAND=$b timeout -k 10 300 bash tools/ab.sh -l base -w headline -s 5 -- --size $sz > /dev/null || exit 1
  done
done
LABEL=base timeout -k 10 300 bash tools/ab.sh -l base -w headline -s 20 > /dev/null || exit 1
cut -c1-120 gpurun_out/ab.log
