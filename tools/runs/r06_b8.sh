# round 6: the whole GPU suite on the current build (pair chains, planner, fetch_directions STOP,
# traceback folds), bench lines, and kernel traces of the headline and local traceback launches
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r6b8_tests.log 2>&1 || { tail -n 40 gpurun_out/r6b8_tests.log; exit 1; }
tail -n 1 gpurun_out/r6b8_tests.log
: > gpurun_out/ab.log
for rep in 1 2; do
  timeout -k 10 600 bash tools/ab.sh -w "headline local dna8k protein4k batch" -s 20 > /dev/null || exit 1
done
cut -c1-200 gpurun_out/ab.log
cp gpurun_out/ab.log gpurun_out/r6b8_ab.log
cd /tmp && export TMPDIR=/tmp
for w in headline local; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r6b8_$w -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r6b8_trace_$w.json 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, os
root = os.environ["GRAFT_REPO_ROOT"]
for w in ("headline", "local"):
    f = glob.glob(f"{root}/gpurun_out/prof_r6b8_{w}/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        if any(k in r["Name"] for k in ("tb_", "expand", "walk", "fill_kernel")):
            print(w, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us")
PY
