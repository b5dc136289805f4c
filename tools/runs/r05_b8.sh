# round-5 check 8: loop alignment (-falign-loops=64) on the round-start sources (al64b) and on HEAD
# (al64h) against base0 and HEAD, same box, three repetitions
mkdir -p gpurun_out
: > gpurun_out/ab.log
for rep in 1 2 3; do
  timeout -k 10 900 bash tools/ab.sh -l "base0 al64b base al64h" -w "headline" -s 20 > /dev/null || exit 1
done
cut -c1-110 gpurun_out/ab.log
