# round-6 final evidence (3/3), on the last build: the full GPU suite, smoke, trace + PMC profiles of
# the two small single pairs (their traceback's strip tables changed), the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6g_tests.log 2>&1 || { tail -30 gpurun_out/r6g_tests.log; exit 1; }
tail -1 gpurun_out/r6g_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6g_smoke.log 2>&1 || { tail gpurun_out/r6g_smoke.log; exit 1; }
tail -1 gpurun_out/r6g_smoke.log
WORKLOADS="dna8k protein4k" timeout -k 10 900 bash tools/profile_all.sh r6g || exit 1
echo final_c done
