# round-4 check 17: cross-group hand-off against the I/O wave's idle poll sleep (SA_IO_SLEEP 0/1/4/8)
mkdir -p gpurun_out
: > gpurun_out/b17.log
for rep in 1 2 3; do
  for sl in 0 1 4 8; do
    for mode in 0 1; do
      echo "sleep$sl mode=$mode " >> gpurun_out/b17.log
      SA_IO_SLEEP=$sl SA_HIP_LIB=$PWD/build_exp/libsa_m0.so timeout -k 10 120 python tools/band_miss.py 32768 $mode 2>/dev/null | grep "^{" >> gpurun_out/b17.log || { echo failed $sl; exit 1; }
    done
  done
done
python3 - <<'PY'
import ast
cur=None
for l in open('gpurun_out/b17.log'):
    l=l.strip()
    if not l.startswith('{'): cur=l; continue
    d=ast.literal_eval(l)
    if 'total_us' in d: print(f"{cur:14s} total {d['total_us']:7.1f} lag_in {d['lag_in_group_ns']:7.1f} cross {d['lag_cross_ns']:7.1f} misses {d['misses_per_band']:6.1f}")
PY
