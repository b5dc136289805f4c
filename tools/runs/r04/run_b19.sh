# round-4 check 19: band L1 touch of the text codes: product (global 6 bodies ahead, local none) vs
# none (t0) vs 4 / 8 in both modes; GPU suite on the product; headline / local bench A/B
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b19_tests.log 2>&1 || { tail -n 40 gpurun_out/b19_tests.log; exit 1; }
tail -n 2 gpurun_out/b19_tests.log
: > gpurun_out/b19.log
for rep in 1 2 3; do
  for lib in prod t0 t4 t8; do
    for mode in 0 1; do
      echo "$lib mode=$mode " >> gpurun_out/b19.log
      SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 120 python tools/band_miss.py 32768 $mode 2>/dev/null | grep "^{" >> gpurun_out/b19.log || { echo failed $lib; exit 1; }
    done
  done
done
python3 - <<'PY'
import ast
cur=None
for l in open('gpurun_out/b19.log'):
    l=l.strip()
    if not l.startswith('{'): cur=l; continue
    d=ast.literal_eval(l)
    if 'total_us' in d: print(f"{cur:12s} total {d['total_us']:7.1f} lag_in {d['lag_in_group_ns']:7.1f} cross {d['lag_cross_ns']:7.1f}")
PY
: > gpurun_out/b19_ab.log
for rep in 1 2; do
  for lib in new t0; do
    for w in headline local dna8k protein4k; do
      if [ $lib = t0 ]; then export SA_HIP_LIB=$PWD/build_exp/libsa_t0.so; else unset SA_HIP_LIB; fi
      timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b19_x.json 2> gpurun_out/b19_x.err || { tail -n 20 gpurun_out/b19_x.err; exit 1; }
      echo "$rep $lib $w $(python tools/show_bench.py gpurun_out/b19_x.json)" >> gpurun_out/b19_ab.log
    done
  done
done
unset SA_HIP_LIB
cut -c1-140 gpurun_out/b19_ab.log
