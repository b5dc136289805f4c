# round 6: unaligned copy-0 text-profile reads for alphabets of more than 4 letters (UNAL): protein
# parity (band fill, config-4 goldens, the 70020-letter reference case), then same-box A/Bs: protein
# with SA_UNAL=0 / default, DNA with the default / SA_UNAL=1, and protein timelines
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_band_fill.py tests/test_gpu_parity.py > gpurun_out/r6b11_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b11_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b11_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  SA_UNAL=0 LABEL=unal0 timeout -k 10 600 bash tools/ab.sh -w "protein4k" -s 20 > /dev/null || exit 1
  LABEL=default timeout -k 10 600 bash tools/ab.sh -w "protein4k headline local dna8k" -s 20 > /dev/null || exit 1
  SA_UNAL=1 LABEL=unal1 timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k" -s 20 > /dev/null || exit 1
done
cut -c1-170 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b11_ab.log
for U in 0 1; do
  SA_UNAL=$U timeout -k 10 120 python tools/timeline.py --n 4096 --m 4096 --protein --letters 20 --mode 0 > gpurun_out/r6b11_tl_u$U.json 2> gpurun_out/r6b11_tl_err.log || { cat gpurun_out/r6b11_tl_err.log; exit 1; }
done
python3 - <<'PY'
import json
for U in (0, 1):
    d = json.load(open(f"gpurun_out/r6b11_tl_u{U}.json"))
    b = d.get("bands", {})
    print("SA_UNAL", U, "strips end", d["last_end_us"], "clk", d["clk_per_step_mean"], "| bands end", b.get("last_end_us"), "clk", b.get("clk_per_step_mean"))
PY
