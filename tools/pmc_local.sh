#!/bin/bash
# PMC passes (separate runs) for the local 32k chain vs 16 short local chains
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
P2="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_INSTS"
for cfg in "1 32768 32768 1" "1 65536 2048 16"; do
  tag=$(echo $cfg | tr ' ' _)
  for pi in 1 2; do
    if [ $pi = 1 ]; then pmc=$P1; else pmc=$P2; fi
    d=$R/gpurun_out/pmcd_${tag}_${pi}
    timeout -s KILL 90 rocprofv3 --pmc $pmc -d $d -o run --output-format csv -- python3 $R/tools/pmc_local.py $cfg > $R/gpurun_out/pmc_${tag}_${pi}.log 2>&1
    f=$(find $d -name "*counter_collection.csv" | head -1)
    cp $f $R/gpurun_out/pmc_${tag}_${pi}.csv
    rm -rf $d
  done
done
