# round-6 final evidence (1/2): full GPU suite, smoke, rocprofv3 trace + WRITE/FETCH PMC of every
# bench workload and the default bench line with its CPU baseline (tools/profile_all.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6f_tests.log 2>&1 || { tail -30 gpurun_out/r6f_tests.log; exit 1; }
tail -1 gpurun_out/r6f_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f_smoke.log 2>&1 || { tail gpurun_out/r6f_smoke.log; exit 1; }
tail -1 gpurun_out/r6f_smoke.log
timeout -k 10 1000 bash tools/profile_all.sh r6f || exit 1
echo final_a done
