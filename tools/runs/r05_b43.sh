# round-5 closing check on the HEAD build: GPU suite, smoke, default bench line
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/b43_tests.log 2>&1 || { tail -30 gpurun_out/b43_tests.log; exit 1; }
tail -1 gpurun_out/b43_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/b43_smoke.log 2>&1 || { tail gpurun_out/b43_smoke.log; exit 1; }
tail -1 gpurun_out/b43_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/b43_bench.json 2> gpurun_out/b43_bench.err || { tail gpurun_out/b43_bench.err; exit 1; }
cat gpurun_out/b43_bench.json
