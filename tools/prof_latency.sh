#!/bin/bash
# kernel + copy trace of the end-to-end alignSequenceGPU latency at 32768^2 (harness latency mode,
# the reference's dummy protein requests: needs scoreMatrices/ in the working directory)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/plat_cwd
python $R/tools/score_matrices.py $R/gpurun_out/plat_cwd
cd $R/gpurun_out/plat_cwd
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/plat -o run --output-format csv -- $R/sequence-alignment-gpu_amd/bin/sa_benchmarks latency global --sizes 32768x32768,8192x8192 --repeats 3 > $R/gpurun_out/plat.log 2>&1
find $R/gpurun_out/plat \( -name "*stats.csv" -o -name "*kernel_trace.csv" -o -name "*memory_copy_trace.csv" \) | while read f; do cp $f $R/gpurun_out/plat_$(basename $f); done
rm -rf $R/gpurun_out/plat $R/gpurun_out/plat_cwd
