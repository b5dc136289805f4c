# round 6: chains of protein-sized alphabets read copy 0 of their text profiles, shifted in registers
# (kArr8A, fill_r1a.hip): the GPU suite, then same-box A/Bs (protein 4096^2 SA_ALIGN=1 / 0; the DNA
# headline against the previous build, whose kernels' code is identical) and protein timelines
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6b13_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b13_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b13_tests.log
: > gpurun_out/ab.log
for rep in 1 2 3; do
  LABEL=align1 timeout -k 10 600 bash tools/ab.sh -w "protein4k" -s 20 > /dev/null || exit 1
  SA_ALIGN=0 LABEL=align0 timeout -k 10 600 bash tools/ab.sh -w "protein4k" -s 20 > /dev/null || exit 1
  timeout -k 10 600 bash tools/ab.sh -l "base prev" -w "headline" -s 20 > /dev/null || exit 1
done
cut -c1-220 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b13_ab.log
for al in 1 0; do
  SA_ALIGN=$al timeout -k 10 300 python tools/timeline.py --protein --n 4096 --m 4096 > gpurun_out/r6b13_tl_align$al.json || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['bands']; print(sys.argv[1], 'strips clk', d['clk_per_step_mean'], 'end', d['last_end_us'], '| bands clk', b['clk_per_step_mean'], 'end', b['last_end_us'])" gpurun_out/r6b13_tl_align$al.json
done
