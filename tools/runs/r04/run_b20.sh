# round-4 check 20: L1 touch of the strips' text codes (s6, s4 bodies ahead) against none (s0x)
mkdir -p gpurun_out
: > gpurun_out/b20.log
for rep in 1 2 3; do
  for lib in s0x s6 s4; do
    for mode in 0 1; do
      echo "$lib mode=$mode " >> gpurun_out/b20.log
      SA_HIP_LIB=$PWD/build_exp/libsa_$lib.so timeout -k 10 120 python tools/band_miss.py 32768 $mode 2>/dev/null | grep "^{" >> gpurun_out/b20.log || { echo failed $lib; exit 1; }
    done
  done
done
python3 - <<'PY'
import ast
cur=None
for l in open('gpurun_out/b20.log'):
    l=l.strip()
    if not l.startswith('{'): cur=l; continue
    d=ast.literal_eval(l)
    if 'total_us' in d: print(f"{cur:12s} total {d['total_us']:7.1f} lag_in {d['lag_in_group_ns']:7.1f} cross {d['lag_cross_ns']:7.1f}")
PY
