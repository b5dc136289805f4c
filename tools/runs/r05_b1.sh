# round-5 check 1: HEAD as restored (GPU suite + bench lines of every workload), the baseline for this round
mkdir -p gpurun_out
NO_TIMELINE=1 WORKLOADS="headline local dna8k protein4k batch" timeout -k 10 1000 bash tools/gpu_check.sh r5b1_notl || exit 1
