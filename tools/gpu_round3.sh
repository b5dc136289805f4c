set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_edge_cases.py -m gpu > gpurun_out/t1.log 2>&1
rc=$?
tail -3 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
for w in headline local dna8k protein4k; do timeout -k 10 120 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 1; done
python - <<'PY'
import json
for w in ["headline","local","dna8k","protein4k"]:
    d=json.loads(open(f"gpurun_out/b_{w}.json").read().strip().splitlines()[-1])
    print(w, d["value"], d["ms_per_step"], d.get("e2e_ms"), d.get("gcups_fill_plus_traceback"))
PY
bash tools/gpu_tl.sh
timeout -k 10 300 python bench.py --workload batch --native --gpus 1 --steps 3 --warmup 1 > gpurun_out/b_native.json 2>gpurun_out/b_native.err && tail -c 600 gpurun_out/b_native.json
