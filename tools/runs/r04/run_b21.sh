# round-4 check 21: which touch pays: none (t0), band only (s0x, the product), strip only (sb), both (s6)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/b21_tests.log 2>&1 || { tail -n 40 gpurun_out/b21_tests.log; exit 1; }
tail -n 2 gpurun_out/b21_tests.log
: > gpurun_out/b21.log
for rep in 1 2 3; do
  for lib in t0 s0x sb s6; do
    for mode in 0 1; do
      echo "$lib mode=$mode " >> gpurun_out/b21.log
      SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 120 python tools/band_miss.py 32768 $mode 2>/dev/null | grep "^{" >> gpurun_out/b21.log || { echo failed $lib; exit 1; }
    done
  done
done
python3 - <<'PY'
import ast
cur=None
for l in open('gpurun_out/b21.log'):
    l=l.strip()
    if not l.startswith('{'): cur=l; continue
    d=ast.literal_eval(l)
    if 'total_us' in d: print(f"{cur:12s} total {d['total_us']:7.1f} lag_in {d['lag_in_group_ns']:7.1f} cross {d['lag_cross_ns']:7.1f}")
PY
for lib in t0 s0x sb s6; do
  SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b21_x.json 2> gpurun_out/b21_x.err || { tail -n 20 gpurun_out/b21_x.err; exit 1; }
  echo "$lib $(python tools/show_bench.py gpurun_out/b21_x.json | cut -c1-120)"
done
