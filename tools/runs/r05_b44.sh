# round-5 check 44: strip feed read after step 10 / 8 (SA_GEN_PF_STEP; product 14), same box, twice
set -o pipefail
rm -f gpurun_out/ab.log
timeout -k 10 900 bash tools/ab.sh -l "eb pf10 pf8 eb pf10 pf8" -w "headline local" -s 10 || exit 1
