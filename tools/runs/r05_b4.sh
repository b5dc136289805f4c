# round-5 check 4: per-quad band LDS addresses with quad-aligned phases: pq2 (publish before the feed
# check), pqx (publish after, as before), pq3 (pq2 + a second feed read after the publish); band tests on
# each, then a same-box A/B against the round-start build (base0)
mkdir -p gpurun_out
ok=""
for lib in pq2 pqx pq3; do
  if SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 300 python -u -m pytest tests/test_band_fill.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b4_$lib.log 2>&1; then
    ok="$ok $lib"; echo "$lib: $(tail -n 1 gpurun_out/r5b4_$lib.log)"
  else
    echo "$lib: FAILED $(grep -m1 -o 'SA_ERR[A-Z_]*: [^\\]*' gpurun_out/r5b4_$lib.log | head -c 200)"
  fi
done
[ -z "$ok" ] && exit 0
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 600 bash tools/ab.sh -l "base0 $ok" -w "headline local dna8k" -s 20 > /dev/null || exit 1
done
cut -c1-110 gpurun_out/ab.log
