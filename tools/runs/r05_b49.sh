# round-5 check 49: two strips / bands per workgroup (SA_WAVES_PER_GROUP=2: fewer waves sharing a
# CU, more cross-group hand-offs) against the default four, small and headline pairs
set -o pipefail
rm -f gpurun_out/ab.log
LABEL=w4 timeout -k 10 600 bash tools/ab.sh -l base -w "dna8k protein4k headline" -s 10 || exit 1
SA_WAVES_PER_GROUP=2 LABEL=w2 timeout -k 10 600 bash tools/ab.sh -l base -w "dna8k protein4k headline" -s 10 || exit 1
LABEL=w4 timeout -k 10 600 bash tools/ab.sh -l base -w "dna8k protein4k" -s 10 || exit 1
SA_WAVES_PER_GROUP=2 LABEL=w2 timeout -k 10 600 bash tools/ab.sh -l base -w "dna8k protein4k" -s 10 || exit 1
