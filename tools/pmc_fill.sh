#!/bin/bash
# SQ stall breakdown of the fill kernel (two PMC passes, each its own rocprofv3 run): where a
# wave's cycles go (issuing / parked at s_waitcnt / issue-stalled) and its instruction mix.
tag=${1:-pmc}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/pmc_$tag
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(--no-cpu-baseline --steps 3 --warmup 1)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --output-format csv -d "$OUT/p1" -o run -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/p1.out" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_BRANCH --output-format csv -d "$OUT/p2" -o run -- python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/p2.out" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fill_kernel" not in r["Kernel_Name"] and "fill_pair" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]][r["Dispatch_Id"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    vals = [sum(v) for v in d.values()]
    print(f"{k:24s} {sum(vals) / len(vals):16.0f}")
PY
