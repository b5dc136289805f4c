# round-6 final check on the last build (staging kernel): the full GPU suite, smoke, the default bench
# line with its CPU baseline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6h_tests.log 2>&1 || { tail -30 gpurun_out/r6h_tests.log; exit 1; }
tail -1 gpurun_out/r6h_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6h_smoke.log 2>&1 || { tail gpurun_out/r6h_smoke.log; exit 1; }
tail -1 gpurun_out/r6h_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r6h_bench_default.json 2> gpurun_out/r6h_bench_default.err || exit 1
tail -c 300 gpurun_out/r6h_bench_default.json
echo final_d done
