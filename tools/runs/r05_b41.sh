# round-5 check 41: pair-packed batch fill at priority 2 (SA_EXP_PAIR_PRIO) under the pipelined
# traceback vs the same build without, three repetitions, same box
set -o pipefail
for rep in 1 2 3; do
  bash tools/ab.sh -l "eb pprio" -w batch -s 20 || exit 1
done
