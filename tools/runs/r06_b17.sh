# round 6: the copy-0 profile test with short texts
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_band_fill.py -k copy0 > gpurun_out/r6b17_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b17_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b17_tests.log
