# round 6 baseline: GPU suite + bench workloads on the HEAD build (no timeline)
NO_TIMELINE=1 bash tools/gpu_check.sh r6b0
