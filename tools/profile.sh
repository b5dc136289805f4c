#!/usr/bin/env bash
# Profiles bench.py on the GPU box (run through gpurun). Three separate rocprofv3 runs, as the
# MI355X guide prescribes: kernel trace + stats, then one PMC pass per TCC byte counter
# (FETCH_SIZE and WRITE_SIZE cannot share a pass). Output: gpurun_out/prof_<tag>/...
#   usage: tools/profile.sh <tag> [bench.py args...]
set -euo pipefail
TAG=${1:-run}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--no-cpu-baseline --steps 5 --warmup 1)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_pmc_write.json" 2> "$OUT/bench_pmc_write.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_pmc_fetch.json" 2> "$OUT/bench_pmc_fetch.err"
echo "profile $TAG done"
