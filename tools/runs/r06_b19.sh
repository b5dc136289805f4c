# round 6: kernel + copy trace of the end-to-end alignSequenceGPU latency (harness latency mode)
timeout -k 10 200 bash tools/prof_latency.sh || exit 1
tail -n 12 gpurun_out/plat.log
