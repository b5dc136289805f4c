#!/bin/bash
# raw progress-stamped timelines (build_exp/libsa_prog.so) for offline analysis
mkdir -p gpurun_out
SA_TL_SAVE=gpurun_out/tl_local32k.npy SA_HIP_LIB=$PWD/build_exp/libsa_prog.so timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 1 > /dev/null 2>&1 &&
SA_TL_SAVE=gpurun_out/tl_global32k.npy SA_HIP_LIB=$PWD/build_exp/libsa_prog.so timeout -k 10 60 python tools/timeline.py --n 32768 --m 32768 --mode 0 > /dev/null 2>&1
