#!/bin/bash
# SQ counters of the traceback kernel (one pass, <= 8 SQ counters) for tools/tb_timing.py
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $ROOT/gpurun_out/tbpmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $ROOT/gpurun_out/tbpmc/p1 -o run -- python3 $ROOT/tools/tb_timing.py > $ROOT/gpurun_out/tbpmc/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $ROOT/gpurun_out/tbpmc/p2 -o run -- python3 $ROOT/tools/tb_timing.py > $ROOT/gpurun_out/tbpmc/p2.log 2>&1 || exit 1
