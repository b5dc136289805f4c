set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "gap_pairs_batched or data_pairs_batched" > gpurun_out/t0.log 2>&1; echo "t0 rc=$?"; tail -3 gpurun_out/t0.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/t1.log 2>&1
rc=$?
tail -5 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
for w in headline local dna8k protein4k; do timeout -k 10 120 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 1; done
python - <<'PY'
import json
for w in ["headline","local","dna8k","protein4k"]:
    d=json.loads(open(f"gpurun_out/b_{w}.json").read().strip().splitlines()[-1])
    print(w, d["value"], d["ms_per_step"], d.get("roofline",{}).get("achieved"), d.get("e2e_ms"))
PY
