# round-5 check 3: bisect the hand-off timeout of the pq build in the multi-pair band test (pf2 alone,
# per-quad alone), then the A/B of whichever libraries pass
mkdir -p gpurun_out
ok=""
for lib in pf2 pqn; do
  if SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 300 python -u -m pytest tests/test_band_fill.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b3_$lib.log 2>&1; then
    ok="$ok $lib"; echo "$lib: $(tail -n 1 gpurun_out/r5b3_$lib.log)"
  else
    echo "$lib: FAILED $(grep -m1 -o 'SA_ERR[A-Z_]*: [^\\]*' gpurun_out/r5b3_$lib.log | head -c 200)"
  fi
done
[ -z "$ok" ] && exit 0
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 600 bash tools/ab.sh -l "base0 $ok" -w "headline local dna8k" -s 20 > /dev/null || exit 1
done
cut -c1-150 gpurun_out/ab.log
