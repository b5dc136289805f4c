# round-4 final check of the committed tree: GPU suite, smoke(), default bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -n 40 gpurun_out/final_tests.log; exit 1; }
tail -n 2 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -n 20 gpurun_out/final_bench.err; exit 1; }
python tools/show_bench.py gpurun_out/final_bench.json
