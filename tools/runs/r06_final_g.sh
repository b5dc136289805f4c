# round-6 final build (single-pair control-word reset): smoke and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6k_smoke.log 2>&1 || { tail gpurun_out/r6k_smoke.log; exit 1; }
tail -1 gpurun_out/r6k_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r6k_bench_default.json 2> gpurun_out/r6k_bench_default.err || exit 1
tail -c 300 gpurun_out/r6k_bench_default.json
