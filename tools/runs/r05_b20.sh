# round-5 check 20: kernel trace of the headline and 8192^2 bench lines (table traceback kernels)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in headline dna8k protein4k; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b20_$w -o run -- python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b20_$w.log 2>&1 || { tail gpurun_out/b20_$w.log; exit 1; }
f=$(find gpurun_out/prof_b20_$w -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | cut -c1-150
done
