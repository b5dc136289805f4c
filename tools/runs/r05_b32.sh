# round-5 check 32: drain only the band rows strip groups read (kFeedsStrips): band tests, then
# same-box A/B of the HEAD build (hb) vs this change (dr1), three repetitions
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_band_fill.py tests/test_gpu_parity.py > gpurun_out/b32_tests.log 2>&1 || { tail -30 gpurun_out/b32_tests.log; exit 1; }
tail -1 gpurun_out/b32_tests.log
for rep in 1 2 3; do
  bash tools/ab.sh -l "hb dr1" -w "headline local dna8k protein4k" || exit 1
done
bash tools/ab.sh -l "hb dr1" -w "headline local" -s 5 -- --size 65536 || exit 1
