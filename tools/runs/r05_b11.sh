# round-5 check 11: local R = 1 planes without STOP (H recomputed along the path by the row walk):
# the whole GPU suite, then same-box bench lines local / headline against base0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5b11_tests.log 2>&1 || { tail -n 40 gpurun_out/r5b11_tests.log; exit 1; }
tail -n 1 gpurun_out/r5b11_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 600 bash tools/ab.sh -l "base0 base" -w "local headline" -s 20 > /dev/null || exit 1
done
cut -c1-150 gpurun_out/ab.log
