# round-4 check 18: band text-code loads: cache policy (sc0 = p1, nt = p2) and an L1 touch 6 / 10
# bodies ahead (t6, t10) against the product loads (base): fill time and lags (band_miss.py)
mkdir -p gpurun_out
: > gpurun_out/b18.log
for rep in 1 2 3; do
  for lib in base p1 p2 t6 t10; do
    for mode in 0 1; do
      echo "$lib mode=$mode " >> gpurun_out/b18.log
      SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 120 python tools/band_miss.py 32768 $mode 2>/dev/null | grep "^{" >> gpurun_out/b18.log || { echo failed $lib; exit 1; }
    done
  done
done
python3 - <<'PY'
import ast
cur=None
for l in open('gpurun_out/b18.log'):
    l=l.strip()
    if not l.startswith('{'): cur=l; continue
    d=ast.literal_eval(l)
    if 'total_us' in d: print(f"{cur:12s} total {d['total_us']:7.1f} lag_in {d['lag_in_group_ns']:7.1f} cross {d['lag_cross_ns']:7.1f}")
PY
