# round-5 check 33: batch steps pipelined two deep (step k's traceback under step k+1's fill) vs the
# synchronous step, three repetitions, same box
set -o pipefail
for rep in 1 2 3; do
  LABEL=pipe1 bash tools/ab.sh -w batch -s 20 || exit 1
  LABEL=pipe0 bash tools/ab.sh -w batch -s 20 -- --batch-pipeline 0 || exit 1
done
